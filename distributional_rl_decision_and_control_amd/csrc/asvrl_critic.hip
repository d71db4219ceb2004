// asvrl_critic.hip -- the IQN critic trunk of AC-IQN (AC_IQN_model.py:410-480) fused on MFMA.
//
// Rows are (sample b, quantile tau) pairs, R = B*N. Per row:
//   c   = relu(Wc cos(tau*pi*k) + bc)            k = 0..63          (cos_embedding, 64 -> 256)
//   h0  = F[b] * c                                F = state features  (observation_processor)
//   h1  = relu(W1 h0 + b1)                                            (hidden_layer, 256 -> 128)
//   h1g = h1 * G[b]                               G = action features (action_encoder)
//   h2  = relu(W2 h1g + b2)                                           (hidden_layer_2, 128 -> 128)
//   q   = wo . h2 + bo                                                (output_layer, 128 -> 1)
//
// Mapping (one wave = 32 rows, v_mfma_f32_32x32x16_bf16): features are the MFMA M dimension and
// rows the N dimension, so a layer's f32 accumulator (lane = row, registers = features) is fed
// to the next layer as its B operand straight from registers -- registers 8s..8s+7 of a 32-row
// block hold features 16s + 8(j>>2) + 4h + (j&3) (h = lane>>5). The weights (A operand) are
// pre-packed on the host into per-lane fragments in exactly that k order (critic_pack.py), one
// 16-B load per lane per MFMA. Nothing between layers touches LDS or HBM.
//
// Modes:
//   FWD    q only (target critic, agent.py:399)
//   TRAIN  forward + quantile-Huber loss vs the target quantiles (agent.py:406-412) + backward:
//          dF (B,256), dG (B,128) reduced over each sample's taus in registers (xor shuffles),
//          and bf16 row-major activations for the weight gradients (dW = dZ^T X, a split-K
//          GEMM on the host side)
//   ACTOR  forward + backward of -mean(q) to the action features only (agent.py:420-425)
//
// The same trunk is IQN_Policy's (IQN_model.py:74-108) without the action encoder (h1g = h1)
// and with an output layer 128 -> A (A <= 32 actions), run as one more MFMA block (the head
// image is padded to 32 rows):
//   IQN_MAX    target pass of train_IQN: q = max_a Q(row, a)                (agent.py:451-452)
//   IQN_TRAIN  forward, gather at the taken action, quantile-Huber loss, backward
//              (agent.py:455-468); the output layer's gradient leaves as a one-hot bf16
//              [R][32] matrix so its weight gradient is one more 32 x 128 MFMA reduction
//   IQN_ACT    act_iqn (agent.py:227-256): mean over K = 32 taus per state, argmax, epsilon-greedy
#include "asvrl_common.h"
#include "asvrl_mfma.h"
#include "asvrl_lds.h"

namespace asvrl {
namespace {

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
                                            const float* Gl, float* wsum = nullptr) {
  constexpr bool IQN = kIqn<MODE>;
  constexpr bool TRAINM = kTrainMode<MODE>;
  const int r = lane & 31, h = lane >> 5;
  const int grow = tile * 32 + r;
  const int b = grow / NT;
  float tau;
  if (MODE == MODE_IQN_ACT && a.taus == nullptr) tau = act_tau(a, grow);
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
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = ks * 16 + 8 * h + j;
      cx[ks][j] = (elem_t)cos_pi_k_tau(tau, k);
    }
    if (TRAINM)
      *reinterpret_cast<frag8*>(bp(a.acts.cos) + static_cast<size_t>(grow) * kNcos + ks * 16 + 8 * h) = cx[ks];
  }
  // BF: the bf16 build's bias-first accumulators (the bias is the MFMA's initial value, no epilogue add)
  // and ReLU on the packed operands (relu_packed) in the modes that keep no f32 activation; TRAIN keeps
  // the bias-after form its part B recomputes bit for bit. F and G are ReLU outputs (>= 0), so
  // relu(F c) = F relu(c) and relu(round(x)) = round(relu(x)): the same operands either way.
  constexpr bool BF = kBiasFirst && !TRAINM;
  frag8 cpk[16], hpk[16];
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    f32x16 acc0[4];
#pragma unroll
    for (int q4 = 0; q4 < 4; ++q4) acc0[q4] = BF ? bias_nat(L.bc, half * 4 + q4, h) : f32x16{};
#pragma unroll
    for (int ks = 0; ks < kNcos / 16; ++ks) {
#pragma unroll
      for (int q4 = 0; q4 < 4; ++q4) acc0[q4] = mfma(WC[((half * 4 + q4) * 4 + ks) * 64 + lane], cx[ks], acc0[q4]);
    }
#pragma unroll
    for (int q4 = 0; q4 < 4; ++q4) {
      const int mb = half * 4 + q4;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        if constexpr (BF) {
          frag8 cp, hp;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float x = acc0[q4][8 * s + j];
            cp[j] = (elem_t)x;
            hp[j] = (elem_t)(static_cast<float>(Fb[feat(mb, 8 * s + j, h)]) * x);
          }
          cpk[mb * 2 + s] = relu_packed(cp);
          hpk[mb * 2 + s] = relu_packed(hp);
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
  f32x16 acc1[4];
#pragma unroll
  for (int mb = 0; mb < 4; ++mb) acc1[mb] = BF ? bias_nat(L.b1, mb, h) : f32x16{};
  mfma_wrows<kC / 16, 4, MODE != MODE_IQN_ACT>(acc1, [&](int mb, int ks) { return W1[(mb * 16 + ks) * 64 + lane]; },
                         [&](int ks) { return hpk[ks]; });
  frag8 h1pk[8], gpk[8];
#pragma unroll
  for (int mb = 0; mb < 4; ++mb) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      if constexpr (BF) {
        frag8 hp, gp;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float x = acc1[mb][8 * s + j];
          hp[j] = (elem_t)x;
          if constexpr (!IQN) gp[j] = (elem_t)(x * Gb[feat(mb, 8 * s + j, h)]);
        }
        h1pk[mb * 2 + s] = relu_packed(hp);
        gpk[mb * 2 + s] = IQN ? h1pk[mb * 2 + s] : relu_packed(gp);   // IQN: no action features
      } else {
        float gv[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int m = feat(mb, 8 * s + j, h);
          float x = acc1[mb][8 * s + j] + L.b1[m];
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
      for (int g = 0; g < 16; ++g) {
        const float x = BF ? acc2[mb][g] : acc2[mb][g] + L.b2[feat(mb, g, h)];
        acc2[mb][g] = x;  // keep z2 for the relu mask
        h2pk[mb * 2 + (g >> 3)][g & 7] = (elem_t)relu(x);
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
    float part = 0.f;
#pragma unroll
    for (int mb = 0; mb < 4; ++mb) {
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        const int m = feat(mb, g, h);
        float x = BF ? acc2[mb][g] : acc2[mb][g] + L.b2[m];
        acc2[mb][g] = x;  // keep z2 for the relu mask
        part += L.wo[m] * relu(x);
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
        dz2pk[mb * 2 + s][j] = (elem_t)dv[j];
        wsa[((mb & 1) * 2 + s) * 8 + j] = dq * hv[j];
      }
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
      float dv[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float h1 = static_cast<float>(h1pk[mb * 2 + s][j]);
        if constexpr (IQN) {   // no action features
          dv[j] = h1 > 0.f ? acc3[mb][8 * s + j] : 0.f;
        } else {
          dv[j] = h1 > 0.f ? acc3[mb][8 * s + j] * G3[feat(mb, 8 * s + j, h)] : 0.f;
          gsa[(mb * 2 + s) * 8 + j] = acc3[mb][8 * s + j] * h1;
        }
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

// ---------------- TRAIN part B, layer 4: dh0 = W1^T dz1; dF[b] = sum_taus dh0 * c; dzc = dh0 * F * 1[c > 0].
// c = relu(Wc cos + bc) is recomputed (bit-identical to part A's) instead of being kept live across
// the layers, which is what lets both parts run two waves per SIMD.
struct CriticLdsB {
  frag8 wc[lds_frags(kFragWC)];
  frag8 w1t[lds_frags(kFragW1)];
  float bc[kC];
};

template <int NT>
__device__ __forceinline__ void critic_tile_b(const CriticArgs& a, const CriticLdsB& L, int tile, int lane,
                                              const elem_t* Fl) {
  const int r = lane & 31, h = lane >> 5;
  const int grow = tile * 32 + r;
  const int b = grow / NT;
  const float tau = a.taus[grow];
  const elem_t* Fb = Fl + (b - tile * 32 / NT) * kC;   // the wave's LDS row of F[b]
  frag8 cx[kNcos / 16];
#pragma unroll
  for (int ks = 0; ks < kNcos / 16; ++ks)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = ks * 16 + 8 * h + j;
      cx[ks][j] = (elem_t)cos_pi_k_tau(tau, k);
    }
  // dz1 as the chained B operand: element j of k-step ks is feature 16ks + 8(j>>2) + 4h + (j&3)
  frag8 dz1pk[8];
  const elem_t* dz1row = bp(a.acts.dz1) + static_cast<size_t>(grow) * kH;
#pragma unroll
  for (int ks = 0; ks < kH / 16; ++ks) {
    const elem4 lo = *reinterpret_cast<const elem4*>(dz1row + ks * 16 + 4 * h);
    const elem4 hi = *reinterpret_cast<const elem4*>(dz1row + ks * 16 + 8 + 4 * h);
    dz1pk[ks] = frag8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  }
  const frag8* W1T = wimg(L.w1t, a.w.w1t_frag);
  const frag8* WCB = wimg(L.wc, a.w.wc_frag);
  // NT = 32 (row_bcast segment sums) spills at 4 blocks per pass; 2 keeps it in registers
  constexpr int BPP = ASVRL_TRAIN_B_BPP32 != 0 && NT == 32 ? ASVRL_TRAIN_B_BPP32 : 4;
#pragma unroll
  for (int half = 0; half < 8 / BPP; ++half) {  // BPP output blocks per pass: 2 * BPP accumulators live
    f32x16 acc0[BPP], acc4[BPP];
#pragma unroll
    for (int q4 = 0; q4 < BPP; ++q4) {
      acc0[q4] = f32x16{};
      acc4[q4] = f32x16{};
    }
#pragma unroll
    for (int ks = 0; ks < kNcos / 16; ++ks)
#pragma unroll
      for (int q4 = 0; q4 < BPP; ++q4) acc0[q4] = mfma(WCB[((half * BPP + q4) * 4 + ks) * 64 + lane], cx[ks], acc0[q4]);
#pragma unroll
    for (int ks = 0; ks < kH / 16; ++ks)
#pragma unroll
      for (int q4 = 0; q4 < BPP; ++q4)
        acc4[q4] = mfma(W1T[((half * BPP + q4) * 8 + ks) * 64 + lane], dz1pk[ks], acc4[q4]);
    float fsa[16 * BPP];   // dh0 * c of this pass, value (q4 * 2 + s) * 8 + j
#pragma unroll
    for (int q4 = 0; q4 < BPP; ++q4) {
      const int mb = half * BPP + q4;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        float dv[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int m = feat(mb, 8 * s + j, h);
          const float x = acc0[q4][8 * s + j] + L.bc[m];
          const float cv = static_cast<float>((elem_t)relu(x));   // part A's bf16 c
          fsa[(q4 * 2 + s) * 8 + j] = acc4[q4][8 * s + j] * cv;
          dv[j] = cv > 0.f ? acc4[q4][8 * s + j] * static_cast<float>(Fb[m]) : 0.f;
        }
        store16(bp(a.acts.dzc) + static_cast<size_t>(grow) * kC + mb * 32 + 16 * s, dv, h);
      }
    }
    // dF[b] over the sample's NT rows: transpose-reduce, lane r then holds values (r % NT) * PER + i
    xreduce<16 * BPP, NT>(fsa, lane);
    constexpr int PER = 16 * BPP / NT;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int v = (r % NT) * PER + i, g = v >> 3;
      const int m = feat(half * BPP + (g >> 1), 8 * (g & 1) + (v & 7), h);
      const size_t o = static_cast<size_t>(b) * kC + m;
      if (a.dF != nullptr) a.dF[o] = fsa[i];
      if (a.dzF != nullptr) bp(a.dzF)[o] = (elem_t)(static_cast<float>(Fb[m]) > 0.f ? fsa[i] : 0.f);   // encoders' relu / mask
    }
  }
}

template <int NT>
__global__ __launch_bounds__(8 * 64) void critic_train_b_kernel(CriticArgs a) {
  __shared__ CriticLdsB L;
  {
    const frag8* gwc = reinterpret_cast<const frag8*>(a.w.wc_frag);
    const frag8* gw1t = reinterpret_cast<const frag8*>(a.w.w1t_frag);
    if constexpr (kWeightsInLds) {
      copy_frags<8 * 64, kFragWC, kElemBytes == 2 ? 16 : 8>(L.wc, gwc, threadIdx.x);
      copy_frags<8 * 64, kFragW1, kElemBytes == 2 ? 16 : 8>(L.w1t, gw1t, threadIdx.x);
    }
    for (int i = threadIdx.x; i < kC; i += 8 * 64) L.bc[i] = a.w.bc[i];
  }
  // this wave's samples' F rows (read per feature after the dzc stores: LDS, not vmcnt-ordered loads)
  __shared__ __attribute__((aligned(16))) elem_t Fs[8 * (32 / NT) * kC];
  const int tile = blockIdx.x * 8 + (threadIdx.x >> 6);
  elem_t* Fw = Fs + (threadIdx.x >> 6) * (32 / NT) * kC;
  if (tile < a.B * NT / 32) stage_features<NT, false, false>(a, tile, threadIdx.x & 63, Fw, nullptr);
  __syncthreads();
  if (tile < a.B * NT / 32) critic_tile_b<NT>(a, L, tile, threadIdx.x & 63, Fw);
}

// One 32-row tile per wave; 8 waves per workgroup (2 per SIMD), 4 when a tile holds several
// samples (N < 32) so the per-wave feature rows still fit next to the weights in LDS.
template <int NT> struct CriticWaves { static constexpr int n = NT == 32 ? 8 : 4; };
// IQN_ACT (the rollout's K = 32 pass, ~20 k tiles): 16 waves share one staged weight image, 4 per SIMD
// (the 150 KB LDS image admits one workgroup per CU, so the wave count per workgroup sets the occupancy;
// 128 VGPRs then, 6 spilled): 137 vs 150 us per launch, IQN iteration 0.370 vs 0.390 ms. The same for
// FWD / IQN_MAX / ACTOR measured neutral to worse (IQN iteration 0.385 ms; ACTOR spills 53).
#ifndef ASVRL_IQN_ACT_WAVES
#define ASVRL_IQN_ACT_WAVES 16
#endif
template <int MODE, int NT> struct ModeWaves { static constexpr int n = CriticWaves<NT>::n; };
template <> struct ModeWaves<MODE_IQN_ACT, 32> { static constexpr int n = ASVRL_IQN_ACT_WAVES; };

template <int MODE, int NT>
__global__ __launch_bounds__((ModeWaves<MODE, NT>::n) * 64) void critic_kernel(CriticArgs a) {
  constexpr int W = ModeWaves<MODE, NT>::n, S = 32 / NT;
  __shared__ typename LdsOf<MODE>::T L;
  using FT = typename FOf<MODE>::T;
  __shared__ __attribute__((aligned(16))) FT Fs[W * S * kC];
  __shared__ __attribute__((aligned(16))) float Gs[kStageG<MODE> ? W * S * kH : 1];
  __shared__ float Ws[MODE == MODE_TRAIN ? W * (kH + 1) : 1];   // per-wave output-layer gradient sums
  const int tile = blockIdx.x * W + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int tiles = a.B * NT / 32;
  FT* Fw = Fs + (threadIdx.x >> 6) * S * kC;
  float* Gw = Gs + (kStageG<MODE> ? (threadIdx.x >> 6) * S * kH : 0);
  if (tile < tiles) stage_features<NT, kStageG<MODE>, kTrainMode<MODE>>(a, tile, lane, Fw, Gw);
  {
    const frag8* gwc = reinterpret_cast<const frag8*>(kFwdOnly<MODE> ? a.w.wc_frag : a.w.w2t_frag);
    const frag8* gw1 = reinterpret_cast<const frag8*>(a.w.w1_frag);
    const frag8* gw2 = reinterpret_cast<const frag8*>(a.w.w2_frag);
    if constexpr (kWeightsInLds) {
      constexpr int CH = kElemBytes == 2 ? 16 : 8;   // fragments in flight per thread
      copy_frags<W * 64, kFragWC, CH>(L.wc, gwc, threadIdx.x);
      copy_frags<W * 64, kFragW1, CH>(L.w1, gw1, threadIdx.x);
      copy_frags<W * 64, kFragW2, CH>(L.w2, gw2, threadIdx.x);
    }
    for (int i = threadIdx.x; i < kC; i += W * 64) L.bc[i] = a.w.bc[i];
    for (int i = threadIdx.x; i < kH; i += W * 64) {
      L.b1[i] = a.w.b1[i];
      L.b2[i] = a.w.b2[i];
      if (!kIqn<MODE>) L.wo[i] = a.w.wo[i];
    }
    if constexpr (kIqn<MODE>) {
      const frag8* gwo = reinterpret_cast<const frag8*>(a.hd.wo_frag);
      for (int i = threadIdx.x; i < kH / 16 * 64; i += W * 64) L.wo_img[i] = gwo[i];
      const int A = a.hd.n_actions;
      if (MODE == MODE_IQN_TRAIN)
        for (int i = threadIdx.x; i < A * kH; i += W * 64) L.wof[i] = (elem_t)a.hd.wo[i];
      for (int i = threadIdx.x; i < kMaxA; i += W * 64) L.bo_a[i] = i < A ? a.hd.bo[i] : 0.f;
    }
  }
  __syncthreads();
  const bool wout = MODE == MODE_TRAIN && a.acts.wout_part != nullptr;
  float* wsum = wout ? Ws + (threadIdx.x >> 6) * (kH + 1) : nullptr;
  if (tile < tiles) {
    critic_tile<MODE, NT>(a, L, tile, lane, Fw, Gw, wsum);
  } else if (wout) {
    for (int i = lane; i < kH + 1; i += 64) wsum[i] = 0.f;
  }
  if (MODE == MODE_TRAIN && wout) {
    // the workgroup's W tile sums in wave order: one [129] partial per workgroup
    __syncthreads();
    for (int i = threadIdx.x; i < kH + 1; i += W * 64) {
      float acc = 0.f;
#pragma unroll
      for (int w = 0; w < W; ++w) acc += Ws[w * (kH + 1) + i];
      a.acts.wout_part[static_cast<size_t>(blockIdx.x) * (kH + 1) + i] = acc;
    }
  }
}

int train_b_grid(int tiles) { return (tiles + 7) / 8; }

int wout_groups(int B, int N) {   // workgroups of the TRAIN launch = groups of wout_part
  const int tiles = B * N / 32;
  const int W = N == 32 ? CriticWaves<32>::n : (N == 16 ? CriticWaves<16>::n : CriticWaves<8>::n);
  return (tiles + W - 1) / W;
}

template <int MODE, int NT>
void launch_mode(const CriticArgs& a, hipStream_t st) {
  constexpr int W = ModeWaves<MODE, NT>::n;
  const int tiles = a.B * NT / 32;
  hipLaunchKernelGGL((critic_kernel<MODE, NT>), dim3((tiles + W - 1) / W), dim3(W * 64), 0, st, a);
}

template <int NT>
void launch_n(int mode, const CriticArgs& a, hipStream_t st) {
  const int tiles = a.B * NT / 32;
  if (mode == MODE_FWD) {
    launch_mode<MODE_FWD, NT>(a, st);
  } else if (mode == MODE_TRAIN) {
    launch_mode<MODE_TRAIN, NT>(a, st);
    hipLaunchKernelGGL((critic_train_b_kernel<NT>), dim3(train_b_grid(tiles)), dim3(8 * 64), 0, st, a);
  } else if (mode == MODE_ACTOR) {
    launch_mode<MODE_ACTOR, NT>(a, st);
  } else if (mode == MODE_IQN_MAX) {
    launch_mode<MODE_IQN_MAX, NT>(a, st);
  } else if (mode == MODE_IQN_TRAIN) {   // part B (layer 4 + dF) is the critic's
    launch_mode<MODE_IQN_TRAIN, NT>(a, st);
    hipLaunchKernelGGL((critic_train_b_kernel<NT>), dim3(train_b_grid(tiles)), dim3(8 * 64), 0, st, a);
  } else if constexpr (NT == 32) {
    launch_mode<MODE_IQN_ACT, 32>(a, st);
  }
}

int launch(int mode, const CriticArgs& a, void* stream) {
  hipStream_t st = as_stream(stream);
  if (a.N == 8) launch_n<8>(mode, a, st);
  else if (a.N == 16) launch_n<16>(mode, a, st);
  else launch_n<32>(mode, a, st);
  return check_launch("asvrl_critic");
}

// ------------------------------------------------------------------ weight packing
// The A-operand fragment images of AsvCriticWeights from the row-major f32 weights: element
// o = ((mb*KS + ks)*64 + lane)*8 + j of an (M x K) image holds W[mb*32 + (lane&31)][col] with
// col = ks*16 + 8h + j for the input-fed layer and ks*16 + 8(j>>2) + 4h + (j&3) for the
// accumulator-fed (chained) layers; h = lane >> 5. One thread per element, all five images.
constexpr int kPackWc = 256 * 64, kPackW1 = 128 * 256, kPackW2 = 128 * 128;
constexpr int kPackTotal = kPackWc + 2 * kPackW1 + 2 * kPackW2;


constexpr int kPackHead = kMaxA * kH;

__global__ __launch_bounds__(256) void pack_kernel(const float* __restrict__ wc, const float* __restrict__ w1,
                                                   const float* __restrict__ w2, AsvCriticWeights w,
                                                   const float* __restrict__ wout, int n_actions, void* wo_frag) {
  int o = blockIdx.x * 256 + threadIdx.x;
  int row, col;
  if (o >= kPackTotal) {                                // IQN output_layer.weight (A x 128), zero rows to 32
    o -= kPackTotal;
    if (wo_frag == nullptr || o >= kPackHead) return;
    frag_rc(o, kH, true, row, col);
    static_cast<elem_t*>(wo_frag)[o] = (elem_t)(row < n_actions ? wout[row * kH + col] : 0.f);
    return;
  }
  if (o < kPackWc) {                                    // cos_embedding.weight (256 x 64)
    frag_rc(o, 64, false, row, col);
    const_cast<elem_t*>(static_cast<const elem_t*>(w.wc_frag))[o] = (elem_t)wc[row * 64 + col];
    return;
  }
  o -= kPackWc;
  if (o < kPackW1) {                                    // hidden_layer.weight (128 x 256)
    frag_rc(o, 256, true, row, col);
    const_cast<elem_t*>(static_cast<const elem_t*>(w.w1_frag))[o] = (elem_t)w1[row * 256 + col];
    return;
  }
  o -= kPackW1;
  if (o < kPackW2) {                                    // hidden_layer_2.weight (128 x 128)
    frag_rc(o, 128, true, row, col);
    const_cast<elem_t*>(static_cast<const elem_t*>(w.w2_frag))[o] = (elem_t)w2[row * 128 + col];
    return;
  }
  o -= kPackW2;
  if (o < kPackW2) {                                    // its transpose
    frag_rc(o, 128, true, row, col);
    const_cast<elem_t*>(static_cast<const elem_t*>(w.w2t_frag))[o] = (elem_t)w2[col * 128 + row];
    return;
  }
  o -= kPackW2;                                         // hidden_layer.weight^T (256 x 128)
  frag_rc(o, 128, true, row, col);
  const_cast<elem_t*>(static_cast<const elem_t*>(w.w1t_frag))[o] = (elem_t)w1[col * 256 + row];
}

int validate(const AsvCriticWeights* w, const AsvCriticIO* io) {
  ASVRL_REQUIRE(w && io && io->taus, "asvrl_critic: null argument");
  ASVRL_REQUIRE(io->F || (io->obs && w->self_w && w->self_b && w->obj_w && w->obj_b),
                "asvrl_critic: needs F, or obs with the encoder weights");
  ASVRL_REQUIRE(io->G || (io->act && w->ae_w && w->ae_b), "asvrl_critic: needs G, or act with the action encoder");
  ASVRL_REQUIRE(!io->obs || io->ld_obs >= 37, "asvrl_critic: ld_obs must cover the packed observation row");
  ASVRL_REQUIRE(w->wc_frag && w->w1_frag && w->w2_frag && w->bc && w->b1 && w->b2 && w->wo && w->bo,
                "asvrl_critic: null weight");
  ASVRL_REQUIRE(io->N == 8 || io->N == 16 || io->N == 32, "asvrl_critic: N must be 8, 16 or 32");
  ASVRL_REQUIRE(io->B >= 0 && (static_cast<int64_t>(io->B) * io->N) % 32 == 0,
                "asvrl_critic: B*N must be a multiple of 32");
  return 0;
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

}  // namespace
}  // namespace asvrl

using namespace asvrl;

extern "C" int asvrl_critic_forward(const AsvCriticWeights* w, const AsvCriticIO* io, void* stream) {
  if (int rc = validate(w, io)) return rc;
  ASVRL_REQUIRE(io->q != nullptr, "asvrl_critic_forward: null q");
  if (io->B == 0) return 0;
  return launch(MODE_FWD, make_args(w, io), stream);
}

extern "C" int asvrl_critic_train(const AsvCriticWeights* w, const AsvCriticIO* io, const AsvCriticActs* acts,
                                  void* stream) {
  if (int rc = validate(w, io)) return rc;
  ASVRL_REQUIRE(io->row_loss && acts && w->w2t_frag && w->w1t_frag, "asvrl_critic_train: null argument");
  ASVRL_REQUIRE(io->q_targets || (io->q_next && io->rewards && io->dones),
                "asvrl_critic_train: needs q_targets or q_next + rewards + dones");
  ASVRL_REQUIRE(acts->cos && acts->h0 && acts->dzc && acts->h1g && acts->dz1 && acts->dz2 &&
                    ((acts->h2 && acts->dq) || acts->wout_part),
                "asvrl_critic_train: null activation buffer (h2 and dq, or wout_part)");
  ASVRL_REQUIRE(io->Np >= 1 && io->kappa > 0.f, "asvrl_critic_train: bad Np/kappa");
  if (io->B == 0) return 0;
  CriticArgs a = make_args(w, io);
  a.gscale = 1.f / (static_cast<float>(io->B) * static_cast<float>(io->Np));
  a.acts = *acts;
  return launch(MODE_TRAIN, a, stream);
}

extern "C" int asvrl_critic_actor_grad(const AsvCriticWeights* w, const AsvCriticIO* io, void* stream) {
  if (int rc = validate(w, io)) return rc;
  ASVRL_REQUIRE(w->w2t_frag && (io->dG || io->dA), "asvrl_critic_actor_grad: needs dG or dA");
  ASVRL_REQUIRE(!io->dA || io->w_ae, "asvrl_critic_actor_grad: dA needs w_ae");
  if (io->B == 0) return 0;
  return launch(MODE_ACTOR, make_args(w, io), stream);
}

extern "C" int asvrl_critic_pack(const float* wc, const float* w1, const float* w2, const AsvCriticWeights* w,
                                 void* stream) {
  ASVRL_REQUIRE(wc && w1 && w2 && w, "asvrl_critic_pack: null argument");
  ASVRL_REQUIRE(w->wc_frag && w->w1_frag && w->w2_frag && w->w2t_frag && w->w1t_frag,
                "asvrl_critic_pack: null fragment buffer");
  hipLaunchKernelGGL(pack_kernel, dim3((kPackTotal + 255) / 256), dim3(256), 0, as_stream(stream), wc, w1, w2, *w,
                     static_cast<const float*>(nullptr), 0, static_cast<void*>(nullptr));
  return check_launch("asvrl_critic_pack");
}

// ------------------------------------------------------------------ IQN

extern "C" int asvrl_iqn_pack(const float* wc, const float* w1, const float* w2, const float* wout,
                              const AsvCriticWeights* w, const AsvIqnHead* head, void* stream) {
  ASVRL_REQUIRE(wc && w1 && w2 && wout && w && head && head->wo_frag, "asvrl_iqn_pack: null argument");
  ASVRL_REQUIRE(w->wc_frag && w->w1_frag && w->w2_frag && w->w2t_frag && w->w1t_frag,
                "asvrl_iqn_pack: null fragment buffer");
  ASVRL_REQUIRE(head->n_actions >= 1 && head->n_actions <= kMaxA, "asvrl_iqn_pack: 1 <= n_actions <= 32");
  const int total = kPackTotal + kPackHead;
  hipLaunchKernelGGL(pack_kernel, dim3((total + 255) / 256), dim3(256), 0, as_stream(stream), wc, w1, w2, *w, wout,
                     head->n_actions, const_cast<void*>(head->wo_frag));
  return check_launch("asvrl_iqn_pack");
}

namespace {

int iqn_validate(const AsvCriticWeights* w, const AsvIqnHead* hd, const AsvIqnIO* io) {
  ASVRL_REQUIRE(w && hd && io, "asvrl_iqn: null argument");
  ASVRL_REQUIRE(io->F || (io->obs && w->self_w && w->self_b && w->obj_w && w->obj_b),
                "asvrl_iqn: needs F, or obs with the encoder weights");
  ASVRL_REQUIRE(!io->obs || io->ld_obs >= 37, "asvrl_iqn: ld_obs must cover the packed observation row");
  ASVRL_REQUIRE(w->wc_frag && w->w1_frag && w->w2_frag && w->bc && w->b1 && w->b2, "asvrl_iqn: null weight");
  ASVRL_REQUIRE(hd->wo_frag && hd->bo && hd->n_actions >= 1 && hd->n_actions <= kMaxA, "asvrl_iqn: bad head");
  ASVRL_REQUIRE(io->N == 8 || io->N == 16 || io->N == 32, "asvrl_iqn: N must be 8, 16 or 32");
  ASVRL_REQUIRE(io->B >= 0 && (static_cast<int64_t>(io->B) * io->N) % 32 == 0, "asvrl_iqn: B*N must be a multiple of 32");
  return 0;
}

CriticArgs iqn_args(const AsvCriticWeights* w, const AsvIqnHead* hd, const AsvIqnIO* io) {
  CriticArgs a{};
  a.w = *w;
  a.hd = *hd;
  a.F = io->F; a.taus = io->taus; a.B = io->B; a.N = io->N; a.Np = io->Np; a.kappa = io->kappa;
  a.obs = io->obs; a.ld_obs = io->ld_obs; a.xb = io->xb;
  a.qn = io->q_next; a.act = io->actions; a.rew = io->rewards; a.don = io->dones; a.ld_rd = io->ld_rd;
  a.gamma = io->gamma; a.q = io->q; a.row_loss = io->row_loss; a.dzF = io->dzF; a.dz_out = io->dz_out;
  a.tile_loss = io->tile_loss; a.loss_scale = io->loss_scale;
  a.act_out = io->act_out; a.ld_act = io->ld_act; a.step_dev = io->step_dev;
  a.eps_spc = io->eps_steps_per_count; a.eps_total = io->eps_total; a.eps_fraction = io->eps_fraction;
  a.eps_initial = io->eps_initial; a.eps_final = io->eps_final; a.seed = io->seed;
  return a;
}

}  // namespace

extern "C" int asvrl_iqn_forward_max(const AsvCriticWeights* w, const AsvIqnHead* head, const AsvIqnIO* io,
                                     void* stream) {
  if (int rc = iqn_validate(w, head, io)) return rc;
  ASVRL_REQUIRE(io->taus && io->q, "asvrl_iqn_forward_max: needs taus and q");
  if (io->B == 0) return 0;
  return launch(MODE_IQN_MAX, iqn_args(w, head, io), stream);
}

extern "C" int asvrl_iqn_train(const AsvCriticWeights* w, const AsvIqnHead* head, const AsvIqnIO* io,
                               const AsvCriticActs* acts, void* stream) {
  if (int rc = iqn_validate(w, head, io)) return rc;
  ASVRL_REQUIRE(io->taus && head->wo && w->w2t_frag && w->w1t_frag && acts, "asvrl_iqn_train: null argument");
  ASVRL_REQUIRE(io->q_next && io->actions && io->rewards && io->dones && io->dz_out,
                "asvrl_iqn_train: needs q_next, actions, rewards, dones and dz_out");
  ASVRL_REQUIRE(acts->cos && acts->h0 && acts->dzc && acts->h1g && acts->dz1 && acts->h2 && acts->dz2,
                "asvrl_iqn_train: null activation buffer");
  ASVRL_REQUIRE(io->Np >= 1 && io->kappa > 0.f, "asvrl_iqn_train: bad Np/kappa");
  if (io->B == 0) return 0;
  CriticArgs a = iqn_args(w, head, io);
  a.gscale = 1.f / (static_cast<float>(io->B) * static_cast<float>(io->Np));
  a.acts = *acts;
  return launch(MODE_IQN_TRAIN, a, stream);
}

extern "C" int asvrl_iqn_act(const AsvCriticWeights* w, const AsvIqnHead* head, const AsvIqnIO* io, void* stream) {
  if (int rc = iqn_validate(w, head, io)) return rc;
  ASVRL_REQUIRE(io->N == 32, "asvrl_iqn_act: K = 32 quantile samples per state");
  ASVRL_REQUIRE(io->act_out && io->ld_act >= 1 && io->eps_total > 0.0 && io->eps_fraction > 0.0,
                "asvrl_iqn_act: needs act_out, ld_act and the epsilon schedule");
  if (io->B == 0) return 0;
  return launch(MODE_IQN_ACT, iqn_args(w, head, io), stream);
}

extern "C" int32_t asvrl_critic_wout_groups(int32_t B, int32_t N) { return wout_groups(B, N); }
