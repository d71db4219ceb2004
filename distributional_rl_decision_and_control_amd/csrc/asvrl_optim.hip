// asvrl_optim.hip -- the optimiser step of the batched learner on gfx950: global-norm
// gradient clipping (torch.nn.utils.clip_grad_norm_(params, 0.5), agent.py:415,426,471,636)
// fused with Adam (optim.Adam(lr=1e-4), agent.py:75-76,98) over ONE flat f32 parameter
// buffer. Two launches per optimizer step regardless of the parameter count:
//   1. sumsq_kernel: kNormBlocks partial sums of g^2 in f64 (one per block), step += 1
//   2. adam_kernel : every block folds the partials in the same fixed order (so all blocks
//      see the identical norm), scales g by min(1, max_norm / (norm + 1e-6)) in place, as
//      clip_grad_norm_ does, then applies Adam with the bias corrections of the new step.
#include "asvrl_adam.h"

namespace asvrl {
namespace {

constexpr int kNormBlocks = 64;
constexpr int kOptThreads = 256;
#ifndef ASVRL_ADAM_PER_THREAD
#define ASVRL_ADAM_PER_THREAD 1
#endif
constexpr int64_t kAdamPer = ASVRL_ADAM_PER_THREAD;   // parameters per thread (grid size), at most 1024 blocks
// the norm partials folded with wave shuffles and one barrier (1) instead of an eight-barrier LDS tree (0)

__global__ __launch_bounds__(kOptThreads) void sumsq_kernel(const float* __restrict__ g, int64_t n,
                                                             double* __restrict__ partial, float* step) {
  double acc = 0.0;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kOptThreads + threadIdx.x; i < n;
       i += static_cast<int64_t>(kNormBlocks) * kOptThreads) {
    const double x = g[i];
    acc += x * x;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, kWave);
  __shared__ double s[kOptThreads / kWave];
  if ((threadIdx.x & (kWave - 1)) == 0) s[threadIdx.x / kWave] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
#pragma unroll
    for (int w = 0; w < kOptThreads / kWave; ++w) t += s[w];
    partial[blockIdx.x] = t;
    if (blockIdx.x == 0) step[0] += 1.f;
  }
}

__global__ __launch_bounds__(kOptThreads) void adam_kernel(float* __restrict__ p, float* __restrict__ g,
                                                            float* __restrict__ m, float* __restrict__ v, int64_t n,
                                                            const double* __restrict__ partial, int nparts,
                                                            const float* __restrict__ step, float lr, float beta1,
                                                            float beta2, float eps, float max_norm,
                                                            float* __restrict__ norm_out, PackTable pk,
                                                            int64_t* __restrict__ counter) {
  __shared__ float s_norm;
  __shared__ double s_red[kOptThreads];
  __shared__ AsvPackSeg s_pk[ASVRL_MAX_PACK_SEGS];
  // this thread's first parameter, its moments and gradient loaded before the norm fold (they do not
  // depend on it: one memory round trip fewer on the launch's critical path)
  const int64_t i0 = static_cast<int64_t>(blockIdx.x) * kOptThreads + threadIdx.x;
  float g0 = 0.f, m0 = 0.f, v0 = 0.f, p0 = 0.f;
  if (i0 < n) {
    g0 = g[i0];
    m0 = m[i0];
    v0 = v[i0];
    p0 = p[i0];
  }
  // the step's bias corrections (two f64 pow) while the norm partials are folded: only the clip needs the norm
  AdamCoef ac = adam_step_scalars(static_cast<double>(step[0]), lr, beta1, beta2);
  {   // the pack table into LDS (read per element below)
    const int* src = reinterpret_cast<const int*>(pk.s);
    int* dst = reinterpret_cast<int*>(s_pk);
    constexpr int kWords = static_cast<int>(sizeof(AsvPackSeg)) / 4 * ASVRL_MAX_PACK_SEGS;
    for (int k = threadIdx.x; k < kWords; k += kOptThreads) dst[k] = src[k];
  }
  {   // thread t folds partials t, t + 256, ... in order, then a fixed tree: the same in every block
    double x = 0.0;
    x = strided_sum<double>(partial, threadIdx.x, nparts, kOptThreads, x);
    // the tree inside each wave by xor shuffles (no barrier), then the four wave sums in order: one barrier
    // instead of eight (AC-IQN step 0.2626 -> 0.2621 ms, profiles/r04af_adam_wave_tree_ab.txt)
#pragma unroll
    for (int off = 1; off < kWave; off <<= 1) x += __shfl_xor(x, off, kWave);
    if ((threadIdx.x & (kWave - 1)) == 0) s_red[threadIdx.x / kWave] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
      double t = 0.0;
#pragma unroll
      for (int w = 0; w < kOptThreads / kWave; ++w) t += s_red[w];
      const float norm = static_cast<float>(sqrt(t));
      s_norm = norm;
      if (blockIdx.x == 0 && norm_out != nullptr) norm_out[0] = norm;
    }
  }
  __syncthreads();
  adam_clip(ac, s_norm, max_norm);
  for (int64_t i = i0; i < n; i += static_cast<int64_t>(gridDim.x) * kOptThreads) {
    const bool first = i == i0;
    float mo = first ? m0 : m[i], vo = first ? v0 : v[i], gi;
    const float pn = adam_elem(ac, beta2, eps, first ? g0 : g[i], mo, vo, first ? p0 : p[i], gi);
    g[i] = gi;
    m[i] = mo;
    v[i] = vo;
    p[i] = pn;
    pack_param_lds(s_pk, pk.n, i, pn);
  }
  if (counter != nullptr && blockIdx.x == 0 && threadIdx.x == 0) counter[0] += 1;
}

}  // namespace
}  // namespace asvrl

using namespace asvrl;

extern "C" int asvrl_adam_clip(float* params, float* grads, float* exp_avg, float* exp_avg_sq, int64_t n,
                               float* step, float lr, float beta1, float beta2, float eps, float max_norm,
                               float* norm_out, double* work, void* stream) {
  ASVRL_REQUIRE(params && grads && exp_avg && exp_avg_sq && step && work, "asvrl_adam_clip: null argument");
  ASVRL_REQUIRE(n >= 0, "asvrl_adam_clip: negative size");
  if (n == 0) return 0;
  hipLaunchKernelGGL(sumsq_kernel, dim3(kNormBlocks), dim3(kOptThreads), 0, as_stream(stream), grads, n, work,
                     step);
  if (int rc = check_launch("asvrl_adam_clip(norm)")) return rc;
  int64_t nb = (n + kAdamPer * kOptThreads - 1) / (kAdamPer * kOptThreads);
  nb = nb < 1 ? 1 : (nb > 1024 ? 1024 : nb);
  hipLaunchKernelGGL(adam_kernel, dim3(static_cast<unsigned>(nb)), dim3(kOptThreads), 0, as_stream(stream), params,
                     grads, exp_avg, exp_avg_sq, n, work, kNormBlocks, step, lr, beta1, beta2, eps, max_norm, norm_out,
                     PackTable{}, static_cast<int64_t*>(nullptr));
  return check_launch("asvrl_adam_clip(step)");
}

extern "C" int asvrl_adam_step(float* params, float* grads, float* exp_avg, float* exp_avg_sq, int64_t n,
                               const float* step, float lr, float beta1, float beta2, float eps, float max_norm,
                               float* norm_out, const double* norm_parts, int32_t nparts, void* stream) {
  ASVRL_REQUIRE(params && grads && exp_avg && exp_avg_sq && step && norm_parts && nparts >= 1,
                "asvrl_adam_step: null argument");
  ASVRL_REQUIRE(n >= 0, "asvrl_adam_step: negative size");
  if (n == 0) return 0;
  int64_t nb = (n + kAdamPer * kOptThreads - 1) / (kAdamPer * kOptThreads);
  nb = nb < 1 ? 1 : (nb > 1024 ? 1024 : nb);
  hipLaunchKernelGGL(adam_kernel, dim3(static_cast<unsigned>(nb)), dim3(kOptThreads), 0, as_stream(stream), params,
                     grads, exp_avg, exp_avg_sq, n, norm_parts, nparts, step, lr, beta1, beta2, eps, max_norm,
                     norm_out, PackTable{}, static_cast<int64_t*>(nullptr));
  return check_launch("asvrl_adam_step");
}

extern "C" int asvrl_adam_step_pack(float* params, float* grads, float* exp_avg, float* exp_avg_sq, int64_t n,
                                    const float* step, float lr, float beta1, float beta2, float eps, float max_norm,
                                    float* norm_out, const double* norm_parts, int32_t nparts, const AsvPackSeg* segs,
                                    int32_t nseg, int64_t* counter, void* stream) {
  ASVRL_REQUIRE(params && grads && exp_avg && exp_avg_sq && step && norm_parts && nparts >= 1,
                "asvrl_adam_step_pack: null argument");
  ASVRL_REQUIRE(n >= 0 && nseg >= 0 && nseg <= ASVRL_MAX_PACK_SEGS && (nseg == 0 || segs != nullptr),
                "asvrl_adam_step_pack: bad size or pack table");
  PackTable t{};
  for (int k = 0; k < nseg; ++k) {
    const AsvPackSeg& g = segs[k];
    ASVRL_REQUIRE(g.image && g.rows >= 1 && g.cols >= 1 && g.nrep >= 1 && g.flat_off >= 0 &&
                      g.flat_off + static_cast<int64_t>(g.rows) * g.cols <= n,
                  "asvrl_adam_step_pack: segment outside the parameters");
    ASVRL_REQUIRE(g.f32 || (g.K % 16 == 0 && g.K >= 16), "asvrl_adam_step_pack: image K must be a multiple of 16");
    t.s[k] = g;
  }
  t.n = nseg;
  if (n == 0) return 0;
  int64_t nb = (n + kAdamPer * kOptThreads - 1) / (kAdamPer * kOptThreads);
  nb = nb < 1 ? 1 : (nb > 1024 ? 1024 : nb);
  hipLaunchKernelGGL(adam_kernel, dim3(static_cast<unsigned>(nb)), dim3(kOptThreads), 0, as_stream(stream), params,
                     grads, exp_avg, exp_avg_sq, n, norm_parts, nparts, step, lr, beta1, beta2, eps, max_norm,
                     norm_out, t, counter);
  return check_launch("asvrl_adam_step_pack");
}

// 2: bf16 MFMA operands, weight images and saved activations (libasvrl.so); 4: f32 (libasvrl_f32.so)
extern "C" int32_t asvrl_operand_bytes(void) { return kElemBytes; }
