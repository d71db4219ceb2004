// asvrl_adam.h -- the per-element clip + Adam update (clip_grad_norm_ then optim.Adam.step(), agent.py:75-76,98,
// 415-416,426) and the weight-image re-pack of asvrl_optim.hip's adam_kernel.
#pragma once
#include "asvrl_common.h"
#include "asvrl_mfma.h"

namespace asvrl {

struct PackTable {
  AsvPackSeg s[ASVRL_MAX_PACK_SEGS];
  int n;
};

// Position of W[row][col] in an (M x K) A-operand fragment image: the inverse of frag_rc
// (asvrl_mfma.h): o = ((mb*KS + ks)*64 + lane)*8 + j with lane = 32h + (row & 31).
__device__ __forceinline__ int64_t frag_pos(int row, int col, int K, bool chained) {
  const int mb = row >> 5, ks = col >> 4, c = col & 15;
  const int h = chained ? ((c >> 2) & 1) : (c >> 3);
  const int j = chained ? (((c >> 3) << 2) | (c & 3)) : (c & 7);
  const int lane = 32 * h + (row & 31);
  return (static_cast<int64_t>(mb) * (K >> 4) + ks) * 512 + lane * 8 + j;
}

// The updated parameter i into every image position a pack table gives it (asvrl_critic_pack /
// asvrl_mlp_pack / asvrl_iqn_pack write the same values from the same f32 weights).
__device__ __forceinline__ void pack_param(const PackTable& t, int64_t i, float p) {
  for (int k = 0; k < t.n; ++k) {
    const AsvPackSeg& g = t.s[k];
    const int64_t u64 = i - g.flat_off;
    if (u64 < 0 || u64 >= static_cast<int64_t>(g.rows) * g.cols) continue;
    const unsigned u = static_cast<unsigned>(u64), cols = static_cast<unsigned>(g.cols);   // 32-bit division
    const int r = static_cast<int>(u / cols), c = static_cast<int>(u - static_cast<unsigned>(r) * cols);
    for (int q = 0; q < g.nrep; ++q) {
      int R = g.row0 + r + q * g.rep_row, Cc = g.col0 + c + q * g.rep_col;
      if (g.transposed) { const int x = R; R = Cc; Cc = x; }
      if (g.f32) static_cast<float*>(g.image)[R] = p;
      else static_cast<elem_t*>(g.image)[frag_pos(R, Cc, g.K, g.chained != 0)] = static_cast<elem_t>(p);
    }
  }
}

// pack_param over a table copied to LDS: the segment scan unrolled, so its reads are issued together instead
// of a scalar-memory round trip per field, segment and element (the kernel-argument table read in a loop)
__device__ __forceinline__ void pack_param_lds(const AsvPackSeg* __restrict__ t, int n, int64_t i, float p) {
#pragma unroll
  for (int k = 0; k < ASVRL_MAX_PACK_SEGS; ++k) {
    if (k >= n) break;
    const AsvPackSeg g = t[k];
    const int64_t u64 = i - g.flat_off;
    if (u64 < 0 || u64 >= static_cast<int64_t>(g.rows) * g.cols) continue;
    const unsigned u = static_cast<unsigned>(u64), cols = static_cast<unsigned>(g.cols);
    const int r = static_cast<int>(u / cols), c = static_cast<int>(u - static_cast<unsigned>(r) * cols);
    for (int q = 0; q < g.nrep; ++q) {
      int R = g.row0 + r + q * g.rep_row, Cc = g.col0 + c + q * g.rep_col;
      if (g.transposed) { const int x = R; R = Cc; Cc = x; }
      if (g.f32) static_cast<float*>(g.image)[R] = p;
      else static_cast<elem_t*>(g.image)[frag_pos(R, Cc, g.K, g.chained != 0)] = static_cast<elem_t>(p);
    }
  }
}

// The step's scalars, computed identically wherever the update runs.
struct AdamCoef {
  float coef, step_size, bc2_sqrt, w1, w2;
};

// the bias corrections of step t (already incremented); the clip coefficient comes later (adam_clip)
__device__ __forceinline__ AdamCoef adam_step_scalars(double t, float lr, float beta1, float beta2) {
  AdamCoef a;
  a.coef = 1.f;
  a.step_size = static_cast<float>(static_cast<double>(lr) / (1.0 - pow(static_cast<double>(beta1), t)));
  a.bc2_sqrt = static_cast<float>(sqrt(1.0 - pow(static_cast<double>(beta2), t)));
  a.w1 = static_cast<float>(1.0 - static_cast<double>(beta1));
  a.w2 = static_cast<float>(1.0 - static_cast<double>(beta2));
  return a;
}

// clip_grad_norm_'s coefficient from the global norm: max_norm / (norm + 1e-6), clamped to 1
__device__ __forceinline__ void adam_clip(AdamCoef& a, float norm, float max_norm) {
  float coef = 1.f;
  if (max_norm > 0.f) {
    coef = max_norm / (norm + 1e-6f);
    coef = coef < 1.f ? coef : 1.f;
  }
  a.coef = coef;
}

__device__ __forceinline__ AdamCoef adam_coef(float norm, double t, float lr, float beta1, float beta2,
                                              float max_norm) {
  AdamCoef a = adam_step_scalars(t, lr, beta1, beta2);
  adam_clip(a, norm, max_norm);
  return a;
}

// one element: g <- clipped g, Adam moments and parameter (torch's single-tensor Adam, no weight decay)
__device__ __forceinline__ float adam_elem(const AdamCoef& a, float beta2, float eps, float g_raw, float& mo, float& vo,
                                           float po, float& g_out) {
  const float gi = g_raw * a.coef;
  g_out = gi;
  const float mi = mo + a.w1 * (gi - mo);          // exp_avg.lerp_(grad, 1 - beta1)
  const float vi = vo * beta2 + a.w2 * gi * gi;    // exp_avg_sq.mul_(beta2).addcmul_(g, g, 1 - beta2)
  mo = mi;
  vo = vi;
  const float denom = sqrtf(vi) / a.bc2_sqrt + eps;
  return po - a.step_size * (mi / denom);         // param.addcdiv_(exp_avg, denom, -step_size)
}

}  // namespace asvrl
