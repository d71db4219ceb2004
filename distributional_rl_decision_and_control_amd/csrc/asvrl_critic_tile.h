// asvrl_critic_tile.h -- one 32-row tile of the IQN critic trunk (AC_IQN_model.py:410-480, IQN_model.py:74-108)
// in one wave: the modes of asvrl_critic.hip's critic_kernel (see that file's header for the mapping),
// shared with asvrl_critic_fused.hip, whose launch runs the target critic's forward (MODE_FWD) for its own
// samples before the update. Included before any fp-contract pragma: the same arithmetic in both files.
#pragma once
#include "asvrl_common.h"
#include "asvrl_mfma.h"
#include "asvrl_lds.h"

namespace asvrl {
namespace {
namespace ctile {

constexpr int kC = 256, kH = 128, kNcos = 64;
enum { MODE_FWD = 0, MODE_TRAIN = 1, MODE_ACTOR = 2, MODE_IQN_MAX = 3, MODE_IQN_TRAIN = 4, MODE_IQN_ACT = 5 };
constexpr int kMaxA = ASVRL_IQN_MAX_ACTIONS;
template <int MODE> constexpr bool kIqn = MODE >= MODE_IQN_MAX;
template <int MODE> constexpr bool kTrainMode = MODE == MODE_TRAIN || MODE == MODE_IQN_TRAIN;
// the Wc image sits in LDS for the forward-only modes; the backward modes keep W2^T there
template <int MODE> constexpr bool kFwdOnly = MODE == MODE_FWD || MODE == MODE_IQN_MAX || MODE == MODE_IQN_ACT;
#ifndef ASVRL_TRAIN_B_BPP32
#define ASVRL_TRAIN_B_BPP32 2
#endif
// Every wave stages its samples' feature rows in LDS in the prologue (F as bf16 for every mode,
// G in f32 for the AC-IQN critic modes), computing them from the observation rows / actions when
// given (the encoders fused into the trunk) or copying F / G. The per-feature reads that follow
// the activation stores then come from LDS: vmcnt counts stores too, so a global load there
// would first wait for every store in flight. One tile per wave (non-persistent launches also
// share the CUs better with a concurrent stream).
template <int MODE> constexpr bool kStageG = !kIqn<MODE>;
constexpr int kSelfF = 56, kSelfIn = 7, kObjF = 40, kObjIn = 5, kObjN = 5, kObsMask = 32;

struct CriticArgs {
  AsvCriticWeights w;
  const float* F;
  const float* G;
  const float* obs;  // packed observation rows (encoders in-kernel) or NULL (F given)
  int64_t ld_obs;
  const float* ain;  // actions for G = action_encoder(a) or NULL (G given)
  int64_t ld_ain;
  void* xb;          // TRAIN: bf16 copy of obs columns 0..31 per sample
  const float* taus;
  const float* qt;  // (B, Np) target quantiles (TRAIN)
  int B, N, Np;
  float kappa, gscale, dq_const;
  float* q;         // (R) optional
  float* row_loss;  // (R) TRAIN
  float* dF;        // (B, 256) optional
  float* dG;        // (B, 128) optional
  AsvCriticActs acts;
  // q_targets = r + gamma * q_next * (1 - d) formed in the loss loop (agent.py:399-400)
  const float* qn;
  const float* rew;
  const float* don;
  int64_t ld_rd;
  float gamma;
  void* dzF;        // (B, 256) bf16: dF * 1[F > 0]
  float* dzG;       // (B, 128): dG * 1[G > 0]
  const float* wae; // (128, 2) action_encoder.weight (ACTOR dA)
  float* dA;        // (B, 2)
  float* tile_loss;  // [tiles] TRAIN: sum(row_loss) * loss_scale; ACTOR: sum(q) * loss_scale, per 32-row tile
  float loss_scale;
  // IQN
  AsvIqnHead hd;
  const float* act;  // IQN_TRAIN: action index of sample b at act[b * ld_rd]
  void* dz_out;      // IQN_TRAIN: bf16 [R][32]
  double* act_out;   // IQN_ACT
  int64_t ld_act;
  const int64_t* step_dev;
  double eps_spc, eps_total, eps_fraction, eps_initial, eps_final;
  uint64_t seed;
};

// per-tile sum of one value per row (lane half 0 holds the rows), one store per tile
__device__ __forceinline__ void tile_sum_store(float v, int lane, float scale, float* dst) {
  v = (lane >> 5) == 0 ? v : 0.f;
  v = seg_sum<32>(v);                       // lane 31: sum of lanes 0..31
  if (lane == 31) *dst = v * scale;
}

// LDS-resident forward weights: fragment images of Wc, W1, W2 (128 KB) + bc, b1, b2, wo.
constexpr int kFragWC = kC * kNcos / 8, kFragW1 = kH * kC / 8, kFragW2 = kH * kH / 8;
// wc holds Wc's image for FWD and W2^T's for TRAIN / ACTOR (which then read Wc from global at the
// top of the tile, before any store, and need W2^T after the activation stores have started)
struct CriticLds {
  frag8 wc[lds_frags(kFragWC)];
  frag8 w1[lds_frags(kFragW1)];
  frag8 w2[lds_frags(kFragW2)];
  float bc[kC], b1[kH], b2[kH], wo[kH];
};
static_assert(kFragWC == kFragW2, "the Wc / W2^T slot holds either image");

// IQN head in LDS: the padded 32 x 128 output image, output_layer.weight in f32 for the
// backward (dh2 = W_out[a] dq) and the bias
struct CriticLdsIqn : CriticLds {
  frag8 wo_img[kH / 16 * 64];
  elem_t wof[kMaxA * kH];   // output_layer.weight (the backward's dh2 = W_out[a] dq feeds a bf16 dz2)
  float bo_a[kMaxA];
};
template <int MODE> struct LdsOf { using T = CriticLds; };
template <> struct LdsOf<MODE_IQN_MAX> { using T = CriticLdsIqn; };
template <> struct LdsOf<MODE_IQN_TRAIN> { using T = CriticLdsIqn; };
template <> struct LdsOf<MODE_IQN_ACT> { using T = CriticLdsIqn; };
// the staged F rows: f32 copies of the operand-rounded values (no per-use conversion) in the AC-IQN
// modes; operand-typed in the IQN modes, whose larger LDS image leaves no room for them
template <int MODE> struct FOf { using T = float; };
template <> struct FOf<MODE_IQN_MAX> { using T = elem_t; };
template <> struct FOf<MODE_IQN_TRAIN> { using T = elem_t; };
template <> struct FOf<MODE_IQN_ACT> { using T = elem_t; };
static_assert(sizeof(CriticLdsIqn) <= 160 * 1024, "IQN LDS image exceeds the CU's 160 KB");

// The wave's feature rows in LDS for its 32 / NT samples: F (bf16 [S][256]) = observation_processor
// of the observation row (AC_IQN_model.py:284-308, IQN_model.py:80-96: self_encoder 7 -> 56 and
// object_encoder 5 -> 40 per object, ReLU, objects with mask < 0.5 zeroed), f32 dot products with
// 4 features per lane, or a copy of a.F; G (f32 [S][128]) = relu(action_encoder(a))
// (AC_IQN_model.py:468-470) or a copy of a.G. TRAIN also writes the bf16 obs copy for the encoder
// weight gradient. Global loads only: this runs before any store of the tile.
template <int NT, bool WITH_G, bool WITH_XB, class FT>
__device__ __forceinline__ void stage_features(const CriticArgs& a, int tile, int lane, FT* Fw, float* Gw) {
  constexpr int S = 32 / NT;
#pragma unroll
  for (int k = 0; k < S; ++k) {
    const int b = tile * S + k;
    if (a.obs != nullptr) {
      const float* x = a.obs + static_cast<int64_t>(b) * a.ld_obs;
      // branch-free (the self / object choice is a per-lane select of the operand addresses), so all
      // four features' loads issue together: one memory round trip instead of two per feature.
      // Same products and summation order as the two-branch form.
      float w[kC / 64][kSelfIn], xs[kC / 64][kSelfIn], bb[kC / 64], mk[kC / 64];
      bool self[kC / 64];
#pragma unroll
      for (int t = 0; t < kC / 64; ++t) {
        const int m = lane + 64 * t;
        self[t] = m < kSelfF;
        const int o = self[t] ? 0 : (m - kSelfF) / kObjF, j = self[t] ? 0 : (m - kSelfF) % kObjF;
        const float* wp = self[t] ? a.w.self_w + m * kSelfIn : a.w.obj_w + j * kObjIn;
        const float* xp = self[t] ? x : x + kSelfIn + kObjIn * o;
#pragma unroll
        for (int i = 0; i < kSelfIn; ++i) {
          const int ii = (i < kObjIn || self[t]) ? i : 0;   // objects read 5 inputs (no read past obj_w)
          w[t][i] = wp[ii];
          xs[t][i] = xp[ii];
        }
        bb[t] = self[t] ? a.w.self_b[m] : a.w.obj_b[j];
        mk[t] = self[t] ? 1.f : x[kObsMask + o];
      }
#pragma unroll
      for (int t = 0; t < kC / 64; ++t) {
        float d = 0.f;
#pragma unroll
        for (int i = 0; i < kSelfIn; ++i)
          if (i < kObjIn || self[t]) d += w[t][i] * xs[t][i];
        const float v = mk[t] < 0.5f ? 0.f : relu(d + bb[t]);   // masked_fill(mask < 0.5, 0)
        Fw[k * kC + lane + 64 * t] = static_cast<FT>((elem_t)v);   // the operand-rounded F (f32 or elem_t)
      }
      if (WITH_XB && a.xb != nullptr && lane < 32) bp(a.xb)[static_cast<int64_t>(b) * 32 + lane] = (elem_t)x[lane];
    } else {
      const float* f = a.F + static_cast<int64_t>(b) * kC;
#pragma unroll
      for (int t = 0; t < kC / 64; ++t) Fw[k * kC + lane + 64 * t] = static_cast<FT>((elem_t)relu(f[lane + 64 * t]));   // ReLU outputs
    }
    if constexpr (WITH_G) {
      if (a.ain != nullptr) {
        const float a0 = a.ain[static_cast<int64_t>(b) * a.ld_ain], a1 = a.ain[static_cast<int64_t>(b) * a.ld_ain + 1];
#pragma unroll
        for (int t = 0; t < kH / 64; ++t) {
          const int m = lane + 64 * t;
          Gw[k * kH + m] = relu((a.w.ae_w[2 * m] * a0 + a.w.ae_w[2 * m + 1] * a1) + a.w.ae_b[m]);
        }
      } else {
#pragma unroll
        for (int t = 0; t < kH / 64; ++t) Gw[k * kH + lane + 64 * t] = relu(a.G[static_cast<int64_t>(b) * kH + lane + 64 * t]);
      }
    }
  }
}

// output-layer weight feeding dh2[m]: the critic's single output row, or IQN's row of the taken action
__device__ __forceinline__ float out_w(const CriticLds& L, int, int m) { return L.wo[m]; }
__device__ __forceinline__ float out_w(const CriticLdsIqn& L, int ai, int m) { return static_cast<float>(L.wof[ai * kH + m]); }

__device__ __forceinline__ uint64_t act_step(const CriticArgs& a) {
  return a.step_dev != nullptr ? static_cast<uint64_t>(*a.step_dev) : 0ull;
}

// act_iqn's quantile fractions when the caller passes none: uniform [0, 1) per row (calc_cos's
// torch.rand, IQN_model.py:63), Philox on (row, step)
__device__ __forceinline__ float act_tau(const CriticArgs& a, int grow) {
  const uint64_t step = act_step(a);
  const U4 u = philox4x32_10(U4{static_cast<uint32_t>(grow), static_cast<uint32_t>(step),
                                static_cast<uint32_t>(step >> 32), 0x1A7u},
                             static_cast<uint32_t>(a.seed), static_cast<uint32_t>(a.seed >> 32));
  return static_cast<float>(u.x >> 8) * (1.0f / 16777216.0f);
}

// act_iqn's selection (agent.py:240-250) for the state of this tile (its 32 rows = the K = 32
// quantile samples): argmax_a of sum_n Q (= K * mean, same argmax; np.argmax's first maximum),
// then greedy iff random() > eps, else a uniform action.
__device__ __forceinline__ void iqn_act_select(const CriticArgs& a, const CriticLdsIqn& L, const f32x16& ao,
                                               int tile, int lane) {
  const int h = lane >> 5, A = a.hd.n_actions;
  float best = -__builtin_inff();
  int bi = kMaxA;
#pragma unroll
  for (int g = 0; g < 16; ++g) {
    const int m = feat(0, g, h);
    float v = m < A ? ao[g] + L.bo_a[m] : 0.f;
    v = seg_sum<32>(v);   // lanes 31 / 63: the sum over the state's 32 taus
    if (m < A && v > best) {
      best = v;
      bi = m;
    }
  }
  const float ob = __shfl_xor(best, 32, 64);
  const int oi = __shfl_xor(bi, 32, 64);
  if (ob > best || (ob == best && oi < bi)) bi = oi;
  if (lane != 31) return;
  // epsilon: linear schedule of the device step counter (trainer.py:257-264)
  const uint64_t step = act_step(a);
  const double progress = static_cast<double>(step) * a.eps_spc / a.eps_total;
  const double eps = progress < a.eps_fraction
                         ? a.eps_initial + (progress / a.eps_fraction) * (a.eps_final - a.eps_initial)
                         : a.eps_final;
  const U4 u = philox4x32_10(U4{static_cast<uint32_t>(tile), static_cast<uint32_t>(step),
                                static_cast<uint32_t>(step >> 32), 0x1A8u},
                             static_cast<uint32_t>(a.seed), static_cast<uint32_t>(a.seed >> 32));
  const double c = (static_cast<double>(u.x >> 8) + 1.0) * (1.0 / 16777216.0);   // random() in (0, 1]
  int act = bi;
  if (!(c > eps)) {   // random.choice(np.arange(action_size))
    act = static_cast<int>((static_cast<uint64_t>(u.y >> 8) * static_cast<uint64_t>(A)) >> 24);
  }
  a.act_out[static_cast<int64_t>(tile) * a.ld_act] = static_cast<double>(act);
}

// acc[mb] += W(mb, ks) B(ks) over ks < KS for MB feature blocks, the weight fragments W (staged in LDS)
// of k-step ks + 1 read while k-step ks's MFMAs issue, one scheduling fence per k-step: otherwise each
// MFMA waits on its own fragment read (A/B knob; same MFMA order, bit-identical). Not for IQN_ACT, whose
// 16-wave launch holds 128 VGPRs.
#ifndef ASVRL_CRIT_READ_AHEAD
#define ASVRL_CRIT_READ_AHEAD 0
#endif
template <int KS, int MB, bool RA, class WF, class BF>
__device__ __forceinline__ void mfma_wrows(f32x16 (&acc)[MB], WF wf, BF bf) {
  if constexpr (ASVRL_CRIT_READ_AHEAD == 0 || !RA) {
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int mb = 0; mb < MB; ++mb) acc[mb] = mfma(wf(mb, ks), bf(ks), acc[mb]);
  } else {
    frag8 aq[2][MB];
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) aq[0][mb] = wf(mb, 0);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      if (ks + 1 < KS)
#pragma unroll
        for (int mb = 0; mb < MB; ++mb) aq[(ks + 1) % 2][mb] = wf(mb, ks + 1);
#pragma unroll
      for (int mb = 0; mb < MB; ++mb) acc[mb] = mfma(aq[ks % 2][mb], bf(ks), acc[mb]);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
}

template <int MODE, int NT, class LT, class FT>
__device__ __forceinline__ void critic_tile(const CriticArgs& a, const LT& L, int tile, int lane, const FT* Fl,
                                            const float* Gl, float* wsum = nullptr, const float* tau_tile = nullptr) {
  constexpr bool IQN = kIqn<MODE>;
  constexpr bool TRAINM = kTrainMode<MODE>;
  const int r = lane & 31, h = lane >> 5;
  const int grow = tile * 32 + r;
  const int b = grow / NT;
  float tau;
  if (MODE == MODE_IQN_ACT && a.taus == nullptr) tau = act_tau(a, grow);
  else if (tau_tile != nullptr) tau = tau_tile[r];   // the tile's taus staged by the caller (LDS)
  else tau = a.taus[grow];
  const FT* Fb = Fl + (b - tile * 32 / NT) * kC;                       // F[b], the wave's LDS row
  const float* Gb = IQN ? nullptr : Gl + (b - tile * 32 / NT) * kH;     // G[b]
  const frag8* WC = kFwdOnly<MODE> ? wimg(L.wc, a.w.wc_frag) : reinterpret_cast<const frag8*>(a.w.wc_frag);
  const frag8* W1 = wimg(L.w1, a.w.w1_frag);
  const frag8* W2 = wimg(L.w2, a.w.w2_frag);

  // ---------------- layer 0: c = relu(Wc cos + bc), h0 = F[b] * c   (two halves of 4 blocks)
  frag8 cx[kNcos / 16];
#pragma unroll
  for (int ks = 0; ks < kNcos / 16; ++ks) {
    float cv[8];
    cos_pi_k_tau8(tau, ks * 16, h, cv);   // k = 16 ks + 8 h + j
    cx[ks] = pack8(cv);
    if (TRAINM)
      *reinterpret_cast<frag8*>(bp(a.acts.cos) + static_cast<size_t>(grow) * kNcos + ks * 16 + 8 * h) = cx[ks];
  }
  // BF: the bf16 build's bias-first accumulators (the bias is the MFMA's initial value, no epilogue add)
  // and ReLU on the packed operands (relu_packed) in the modes that keep no f32 activation; TRAIN keeps
  // the bias-after form its part B recomputes bit for bit. F and G are ReLU outputs (>= 0), so
  // relu(F c) = F relu(c) and relu(round(x)) = round(relu(x)): the same operands either way.
  constexpr bool BF = kBiasFirst && !TRAINM;
  // QB of the eight 32-feature blocks per pass: four, or two in the 16-wave IQN_ACT launch, whose 128
  // VGPRs then hold one pass's accumulators beside the packed outputs of the passes before it (the same
  // MFMAs per block in the same k order: bit-identical)
  constexpr int QB = MODE == MODE_IQN_ACT ? 2 : 4;
  frag8 cpk[16], hpk[16];
#pragma unroll
  for (int half = 0; half < 8 / QB; ++half) {
    f32x16 acc0[QB];
#pragma unroll
    for (int q4 = 0; q4 < QB; ++q4) acc0[q4] = BF ? bias_nat(L.bc, half * QB + q4, h) : f32x16{};
#pragma unroll
    for (int ks = 0; ks < kNcos / 16; ++ks) {
#pragma unroll
      for (int q4 = 0; q4 < QB; ++q4) acc0[q4] = mfma(WC[((half * QB + q4) * 4 + ks) * 64 + lane], cx[ks], acc0[q4]);
    }
#pragma unroll
    for (int q4 = 0; q4 < QB; ++q4) {
      const int mb = half * QB + q4;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        if constexpr (BF) {
          float xs[8], fs[8], hs[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            xs[j] = acc0[q4][8 * s + j];
            fs[j] = static_cast<float>(Fb[feat(mb, 8 * s + j, h)]);
          }
          mul8(fs, xs, hs);
          cpk[mb * 2 + s] = relu_packed(pack8(xs));
          hpk[mb * 2 + s] = relu_packed(pack8(hs));
        } else {
          float hv[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int m = feat(mb, 8 * s + j, h);
            float x = acc0[q4][8 * s + j] + L.bc[m];
            x = relu(x);
            cpk[mb * 2 + s][j] = (elem_t)x;
            hv[j] = static_cast<float>(Fb[m]) * x;
            hpk[mb * 2 + s][j] = (elem_t)hv[j];
          }
          if (TRAINM)
            store16(bp(a.acts.h0) + static_cast<size_t>(grow) * kC + mb * 32 + 16 * s, hv, h);
        }
      }
    }
  }

  // ---------------- layer 1: h1 = relu(W1 h0 + b1), h1g = h1 * G[b]
  // in passes of QB1 blocks (two in IQN_ACT, for its 128 VGPRs; same per-block k order: bit-identical)
  constexpr int QB1 = MODE == MODE_IQN_ACT ? 2 : 4;
  frag8 h1pk[8], gpk[8];
#pragma unroll
  for (int pass = 0; pass < 4 / QB1; ++pass) {
    f32x16 acc1[QB1];
#pragma unroll
    for (int q = 0; q < QB1; ++q) acc1[q] = BF ? bias_nat(L.b1, pass * QB1 + q, h) : f32x16{};
    mfma_wrows<kC / 16, QB1, MODE != MODE_IQN_ACT>(
        acc1, [&](int q, int ks) { return W1[((pass * QB1 + q) * 16 + ks) * 64 + lane]; }, [&](int ks) { return hpk[ks]; });
#pragma unroll
    for (int q = 0; q < QB1; ++q) {
      const int mb = pass * QB1 + q;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        if constexpr (BF) {
          float xs[8], gs[8], ps[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            xs[j] = acc1[q][8 * s + j];
            if constexpr (!IQN) gs[j] = Gb[feat(mb, 8 * s + j, h)];
          }
          if constexpr (!IQN) mul8(xs, gs, ps);
          h1pk[mb * 2 + s] = relu_packed(pack8(xs));
          gpk[mb * 2 + s] = IQN ? h1pk[mb * 2 + s] : relu_packed(pack8(ps));   // IQN: no action features
        } else {
          float gv[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int m = feat(mb, 8 * s + j, h);
            float x = acc1[q][8 * s + j] + L.b1[m];
            x = relu(x);
            h1pk[mb * 2 + s][j] = (elem_t)x;
            gv[j] = IQN ? x : x * Gb[m];   // IQN: no action features
            gpk[mb * 2 + s][j] = (elem_t)gv[j];
          }
          if (TRAINM)
            store16(bp(a.acts.h1g) + static_cast<size_t>(grow) * kH + mb * 32 + 16 * s, gv, h);
        }
      }
    }
  }

  // ---------------- layer 2: h2 = relu(W2 h1g + b2), q = wo . h2 + bo
  f32x16 acc2[4];
#pragma unroll
  for (int mb = 0; mb < 4; ++mb) acc2[mb] = BF ? bias_nat(L.b2, mb, h) : f32x16{};
  mfma_wrows<kH / 16, 4, MODE != MODE_IQN_ACT>(acc2, [&](int mb, int ks) { return W2[(mb * 8 + ks) * 64 + lane]; },
                         [&](int ks) { return gpk[ks]; });
  float q;
  int ai = 0;   // IQN_TRAIN: the sample's action
  if constexpr (IQN) {
    // output layer 128 -> A as one 32-row MFMA block fed from h2 in registers
    frag8 h2pk[8];
#pragma unroll
    for (int mb = 0; mb < 4; ++mb) {
#pragma unroll
      for (int s8 = 0; s8 < 2; ++s8) {
        float xv[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int g = 8 * s8 + j;
          const float x = BF ? acc2[mb][g] : acc2[mb][g] + L.b2[feat(mb, g, h)];
          acc2[mb][g] = x;  // keep z2 for the relu mask
          xv[j] = x;
        }
        h2pk[mb * 2 + s8] = relu_packed(pack8(xv));   // relu(round(x)) = round(relu(x)), two per instruction
      }
    }
    f32x16 ao = f32x16{};
#pragma unroll
    for (int ks = 0; ks < kH / 16; ++ks) ao = mfma(L.wo_img[ks * 64 + lane], h2pk[ks], ao);
    const int A = a.hd.n_actions;   // register g of half h holds action feat(0, g, h)
    if constexpr (MODE == MODE_IQN_ACT) {
      iqn_act_select(a, L, ao, tile, lane);
      return;
    }
    if constexpr (MODE == MODE_IQN_MAX) {
      float mx = -__builtin_inff();
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        const int m = feat(0, g, h);
        if (m < A) mx = fmaxf(mx, ao[g] + L.bo_a[m]);
      }
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      if (h == 0) a.q[grow] = mx;
      return;
    }
    ai = static_cast<int>(a.act[static_cast<int64_t>(b) * a.ld_rd]);
    ai = ai < 0 ? 0 : (ai >= A ? A - 1 : ai);
    float qs = 0.f;
#pragma unroll
    for (int g = 0; g < 16; ++g)
      if (feat(0, g, h) == ai) qs = ao[g] + L.bo_a[ai];
    q = half_sum(qs);   // Q_expected.gather(2, actions) (agent.py:456): one half holds it, the other 0
  } else {
    // the products two per v_pk_mul_f32, the sum in the same serial order
    float part = 0.f;
#pragma unroll
    for (int mb = 0; mb < 4; ++mb) {
#pragma unroll
      for (int s8 = 0; s8 < 2; ++s8) {
        float wv[8], hv[8], pr[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int g = 8 * s8 + j, m = feat(mb, g, h);
          const float x = BF ? acc2[mb][g] : acc2[mb][g] + L.b2[m];
          acc2[mb][g] = x;  // keep z2 for the relu mask
          wv[j] = L.wo[m];
          hv[j] = relu(x);
        }
        mul8(wv, hv, pr);
#pragma unroll
        for (int j = 0; j < 8; ++j) part += pr[j];
      }
    }
    q = half_sum(part) + a.w.bo[0];
  }
  if (a.q != nullptr && h == 0) a.q[grow] = q;
  if (MODE == MODE_FWD) return;

  // ---------------- dL/dq
  float dq;
  if (TRAINM) {
    const float* qt = a.qn != nullptr ? a.qn + static_cast<size_t>(b) * a.Np : a.qt + static_cast<size_t>(b) * a.Np;
    float rb = 0.f, nd = 0.f;
    if (a.qn != nullptr) {
      rb = a.rew[b * a.ld_rd];
      nd = 1.0f - a.don[b * a.ld_rd];
    }
    // quantile-Huber terms over the target quantiles (agent.py:406-412), each lane half taking
    // half of them; |tau - 1[d < 0]| is tau or 1 - tau (exact), and the division by kappa
    // happens once per row
    const float kap = a.kappa, hk = 0.5f * a.kappa, omt = 1.f - tau;
    float wl = 0.f, wg = 0.f;
    auto term = [&](float target) {
      const float d = target - q;  // td_error (agent.py:406)
      const float ad = fabsf(d);
      const bool quad = ad <= kap;
      const float hub = quad ? 0.5f * (d * d) : kap * (ad - hk);
      const float w = d < 0.f ? omt : tau;
      wl += w * hub;
      wg += w * (quad ? d : copysignf(kap, d));
    };
    if (a.Np == NT) {
      // N' = N: lane r owns target r % N of its sample (one load per lane, no load in the loop);
      // the loop broadcasts it: readlane when one sample fills the 32-row tile, else a shuffle
      const float qv = qt[r % NT];
      const float own = a.qn != nullptr ? rb + (a.gamma * qv) * nd : qv;   // r + gamma * q_next * (1 - d)
#pragma unroll 4
      for (int j = 0; j < NT / 2; ++j) {
        float target;
        if (NT == 32) {
          const float t0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(own), j));
          const float t1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(own), j + NT / 2));
          target = h ? t1 : t0;
        } else {
          target = __shfl(own, (lane & ~(NT - 1)) + j + h * (NT / 2), 64);
        }
        term(target);
      }
    } else {
      for (int j = h; j < a.Np; j += 2) term(a.qn != nullptr ? rb + (a.gamma * qt[j]) * nd : qt[j]);
    }
    wl = half_sum(wl) / kap;
    wg = half_sum(wg) / kap;
    dq = -wg * a.gscale;
    if (a.tile_loss != nullptr) tile_sum_store(wl, lane, a.loss_scale, a.tile_loss + tile);
    if (h == 0) {
      if (a.row_loss != nullptr) a.row_loss[grow] = wl;
      if (a.acts.dq != nullptr) a.acts.dq[grow] = dq;
    }
    if constexpr (MODE == MODE_IQN_TRAIN) {   // dL/d(output pre-activation): dq at the taken action
      frag8 o0, o1;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        o0[i] = (elem_t)(16 * h + i == ai ? dq : 0.f);
        o1[i] = (elem_t)(16 * h + 8 + i == ai ? dq : 0.f);
      }
      elem_t* od = bp(a.dz_out) + static_cast<size_t>(grow) * kMaxA + 16 * h;
      *reinterpret_cast<frag8*>(od) = o0;
      *reinterpret_cast<frag8*>(od + 8) = o1;
    }
  } else {
    dq = a.dq_const;
    if (a.tile_loss != nullptr) tile_sum_store(q, lane, a.loss_scale, a.tile_loss + tile);
  }

  // ---------------- dz2 = dq * wo * 1[z2 > 0]
  // AC-IQN TRAIN with wout_part: output_layer's weight gradient sum_rows dq * h2 is reduced over the
  // tile's 32 rows right here (transpose-reduce per two 32-feature blocks) and then over the
  // workgroup's tiles in LDS, so h2 never goes to HBM
  const bool wout = MODE == MODE_TRAIN && wsum != nullptr;   // this wave's row of the workgroup's LDS sums
  float* wp = wsum;
  frag8 dz2pk[8];
  float wsa[32];
#pragma unroll
  for (int mb = 0; mb < 4; ++mb) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      float hv[8], dv[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int m = feat(mb, 8 * s + j, h);
        const float z = acc2[mb][8 * s + j];
        hv[j] = relu(z);
        dv[j] = z > 0.f ? dq * out_w(L, ai, m) : 0.f;
        wsa[((mb & 1) * 2 + s) * 8 + j] = dq * hv[j];
      }
      dz2pk[mb * 2 + s] = pack8(dv);
      if (TRAINM) {
        const size_t o = static_cast<size_t>(grow) * kH + mb * 32 + 16 * s;
        if (!wout) store16(bp(a.acts.h2) + o, hv, h);
        store16(bp(a.acts.dz2) + o, dv, h);
      }
    }
    if (MODE == MODE_TRAIN && (mb & 1) && wout) {   // wave-uniform
      xreduce<32, 32>(wsa, lane);   // lane r: the tile sum of value r of this block pair
      const int mbb = (mb & ~1) + (r >> 4);
      wp[feat(mbb, 8 * ((r >> 3) & 1) + (r & 7), h)] = wsa[0];
    }
  }
  if (MODE == MODE_TRAIN && wout) {
    const float db = seg_sum<32>(h == 0 ? dq : 0.f);   // lane 31: the tile's sum of dq
    if (lane == 31) wp[kH] = db;
  }

  // ---------------- layer 3: dh1g = W2^T dz2; dG[b] = sum_taus dh1g * h1; dz1 = dh1g * G * 1[h1 > 0]
  const frag8* W2T = wimg(L.wc, a.w.w2t_frag);   // TRAIN / ACTOR stage W2^T in this slot
  f32x16 acc3[4];
#pragma unroll
  for (int mb = 0; mb < 4; ++mb) acc3[mb] = f32x16{};
  mfma_wrows<kH / 16, 4, MODE != MODE_IQN_ACT>(acc3, [&](int mb, int ks) { return W2T[(mb * 8 + ks) * 64 + lane]; },
                         [&](int ks) { return dz2pk[ks]; });
  // dz1 = dh1g * G * 1[h1 > 0]; gsa collects dh1g * h1 for dG = its sum over the sample's taus.
  // G is re-read here through an opaque offset: reusing layer 1's reads would keep 64 values live
  int g0 = 0;
  asm volatile("" : "+v"(g0));
  const float* G3 = Gb + g0;
  float gsa[64];   // value (mb * 2 + s) * 8 + j
#pragma unroll
  for (int mb = 0; mb < 4; ++mb) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      float dv[8], d3[8], h1[8], gh[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        h1[j] = static_cast<float>(h1pk[mb * 2 + s][j]);
        d3[j] = acc3[mb][8 * s + j];
        if constexpr (IQN) {   // no action features
          dv[j] = h1[j] > 0.f ? d3[j] : 0.f;
        } else {
          dv[j] = h1[j] > 0.f ? d3[j] * G3[feat(mb, 8 * s + j, h)] : 0.f;
        }
      }
      if constexpr (!IQN) {
        mul8(d3, h1, gh);
#pragma unroll
        for (int j = 0; j < 8; ++j) gsa[(mb * 2 + s) * 8 + j] = gh[j];
      }
      if (TRAINM)
        store16(bp(a.acts.dz1) + static_cast<size_t>(grow) * kH + mb * 32 + 16 * s, dv, h);
    }
  }
  if constexpr (!IQN) {
    // dG[b] over the sample's NT rows: transpose-reduce, lane r then holds features of values
    // (r % NT) * PER + i
    xreduce<64, NT>(gsa, lane);
    constexpr int PER = 64 / NT;
    float pa0 = 0.f, pa1 = 0.f;   // ACTOR: partial dA over this lane's features
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int v = (r % NT) * PER + i, g = v >> 3;
      const int m = feat(g >> 1, 8 * (g & 1) + (v & 7), h);
      const float gm = G3[m];
      const float gz = gm > 0.f ? gsa[i] : 0.f;   // through the action encoder's relu
      const size_t o = static_cast<size_t>(b) * kH + m;
      if (a.dG != nullptr) a.dG[o] = gsa[i];
      if (a.dzG != nullptr) a.dzG[o] = gz;
      if (MODE == MODE_ACTOR && a.dA != nullptr) {
        pa0 += gz * a.wae[2 * m];
        pa1 += gz * a.wae[2 * m + 1];
      }
    }
    if (MODE == MODE_ACTOR && a.dA != nullptr) {
      pa0 = half_sum(seg_sum<NT>(pa0));   // lane r % NT == NT - 1 of each half holds the group sum
      pa1 = half_sum(seg_sum<NT>(pa1));
      if ((r % NT) == NT - 1 && h == 0) {
        a.dA[2 * b] = pa0;
        a.dA[2 * b + 1] = pa1;
      }
    }
  }
}

CriticArgs make_args(const AsvCriticWeights* w, const AsvCriticIO* io) {
  CriticArgs a{};
  a.w = *w;
  a.F = io->F; a.G = io->G; a.taus = io->taus; a.B = io->B; a.N = io->N; a.Np = io->Np; a.kappa = io->kappa;
  a.obs = io->obs; a.ld_obs = io->ld_obs; a.ain = io->act; a.ld_ain = io->ld_act; a.xb = io->xb;
  a.qt = io->q_targets; a.qn = io->q_next; a.rew = io->rewards; a.don = io->dones; a.ld_rd = io->ld_rd;
  a.gamma = io->gamma; a.dq_const = io->dq; a.q = io->q; a.row_loss = io->row_loss; a.dF = io->dF; a.dG = io->dG;
  a.dzF = io->dzF; a.dzG = io->dzG; a.wae = io->w_ae; a.dA = io->dA;
  a.tile_loss = io->tile_loss; a.loss_scale = io->loss_scale;
  return a;
}

}  // namespace ctile
}  // namespace
}  // namespace asvrl
