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
#include "asvrl_critic_tile.h"

namespace asvrl {
namespace {

using namespace ctile;

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
