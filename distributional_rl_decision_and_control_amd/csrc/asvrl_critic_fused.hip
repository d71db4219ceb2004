// asvrl_critic_fused.hip -- the critic update of train_AC_IQN (agent.py:395-414) with its weight
// gradients in ONE persistent launch: forward, quantile-Huber loss, backward AND the per-workgroup
// reductions dW = dZ^T X of every trunk layer, so no activation ever goes to HBM.
//
// Per row (sample b, quantile tau), the trunk of AC_IQN_model.py:410-480 (see asvrl_critic.hip):
//   c = relu(Wc cos(tau pi k) + bc), x = F[b] * c, h1 = relu(W1 x + b1), h1g = h1 * G[b],
//   z2 = W2 h1g + b2, q = wo . relu(z2) + bo.
//
// Work split (one workgroup per CU, 4 waves = one per SIMD, 512 registers each): the workgroup takes
// ROUNDS of G = 32 NB rows; inside a round the four waves split every layer's OUTPUT FEATURES
// (wave w: cos-layer features 64w..64w+63, hidden features 32w..32w+31) for all G rows, and exchange
// the layer outputs through LDS. The weight-gradient reduction over rows then needs no second copy
// of anything: wave w owns dW rows of its own features, dW[own][:] += dZ[:, own]^T X (A operand =
// its own dZ slice, B operand = the whole X image, both read transposed with ds_read_b64_tr_b16),
// and keeps those accumulators (dW2 32x128, dW1 32x256, dWc 64x64 = 256 registers) for its whole
// life. At the end each workgroup writes one [M*K + M] partial per layer (asvrl_partial_sums sums the
// workgroups in a fixed order: deterministic).
//
// LDS images hold activations in "chained position" order: position p of a 32-feature block is
// feature p with bits 2 and 3 swapped, which is exactly the k order of the pre-packed chained weight
// fragments (asvrl_mfma.h) and the register order of an accumulator block: a lane's 8 registers of
// one k-group are 8 consecutive positions (one 16-byte store), and a B-operand fragment of the next
// layer is one 16-byte load. Rows are XOR-swizzled so that both the row reads (ds_read_b128, 16 rows
// per lane group) and the transposed reads (4 rows x 64 B per 32-lane half) are bank-conflict free.
//
// Weights (A operands) are read from the global fragment images (L2-resident, every workgroup reads
// the same 224 KB) and reused over the NB row blocks of a round.
//
// Per round: stage (F, G, cos) | L0 -> x | L1 -> h1g | L2 -> q partials | loss -> dq | dz2, dwo |
// dW2 + L3 (W2^T dz2) -> dG, dz1 | dW1 | L4 (W1^T dz1, c recomputed) -> dF, dzc | dWc, ten barriers.
//
// IQN (template flag; train_IQN, agent.py:449-468, IQN_model.py:74-108): the same trunk without the
// action encoder (h1g = h1, no G / dG), q = W_out[a_b] . h2 + b_out[a_b] at the sample's action, and the
// output layer's gradient as one more MFMA per wave and round, dW_out[:, own] += D^T h2 with D the
// one-hot dq image (rows = 32 padded actions), accumulated in VGPRs.
#include "asvrl_common.h"
#include "asvrl_mfma.h"
#include "asvrl_lds.h"
// the target critic's forward inside this launch (target_phase) runs at one wave per SIMD, where nothing hides an
// MFMA's wait for its weight fragment: read each k-step's fragments one step ahead (same MFMAs in the same order,
// bit-identical; TQ launch 136 -> 130 us, step 0.2545 -> 0.2500 ms, profiles/r05ae_tq_read_ahead_ab.txt). The
// separate forward launch (two waves per SIMD) keeps asvrl_critic_tile.h's default, measured neutral there.
#ifndef ASVRL_CRIT_READ_AHEAD
#define ASVRL_CRIT_READ_AHEAD 1
#endif
#include "asvrl_critic_tile.h"   // before the contraction pragma: the target critic's forward as asvrl_critic.hip's

// FMA contraction of this file's f32 epilogue arithmetic (the loss terms, the output layer's and the encoders'
// gradient sums, the Bellman target): one v_fma_f32 where the source writes a * b + c (the library is built
// with -ffp-contract=off for the env kernel's f64 parity). stage_fg's encoder dot products stay uncontracted,
// op for op what oracle/learn_ref.critic_step_bf16 restates.
#ifndef ASVRL_FUSED_CONTRACT
#define ASVRL_FUSED_CONTRACT 1
#endif
#if ASVRL_FUSED_CONTRACT
#pragma clang fp contract(fast)
#endif

namespace asvrl {
namespace {

constexpr int kC = 256, kH = 128, kNcos = 64, kNW = 4, kMaxA = ASVRL_IQN_MAX_ACTIONS;

// a round issues the global loads of the next round's inputs behind the W2 fragment fetch in L1, so the
// wait for the weight fragments fetched before it never includes these loads (127-129 vs 130 us per launch
// against issuing them at the top of the round, stage phase 3.7k -> 3.1k cycles: profiles/r02_enc_ab.txt)
// stage-ahead (1, default): round t + grid's F, G and cos images are staged in round t's last phase,
// behind the dW1 MFMAs, into a second set of images (double-buffered), so a round starts with its first
// layer instead of the staging phase and its barrier. Where the second set fits in LDS: AC-IQN, N = 32,
// bf16 operands (the bench shape). Measured 129-133 -> 125-127 us per launch, round 34.2k -> 33.4k
// cycles (profiles/r02_stage_ahead_ab.txt).
#ifndef ASVRL_STAGE_AHEAD
#define ASVRL_STAGE_AHEAD 1
#endif
// stage-ahead for IQN_Policy's update at N = 32 too (its second image set fits: no action features):
// IQN loop 2852-2863 -> 2892-2896 learn-steps/s (profiles/r02_iqn_stage_ahead_ab.txt)
#ifndef ASVRL_STAGE_AHEAD_IQN
#define ASVRL_STAGE_AHEAD_IQN 1
#endif
// with stage-ahead: the cos layer's weight fragments of the wave's two blocks held in registers for the
// kernel's life (L0 and L4 read the same 8 fragments every round) instead of fetched three times a round
// (the VGPRs stage-ahead frees): 125-127 -> 121-126 us, round 32.8k cycles (profiles/r02_wc_resident_ab.txt)
#ifndef ASVRL_WC_RESIDENT
#define ASVRL_WC_RESIDENT 1
#endif

#if ASVRL_OPERAND_F32
template <int NT> struct FusedNB { static constexpr int v = 1; };
#else
template <int NT> struct FusedNB { static constexpr int v = 2; };
#endif

// keep a fragment materialised in its packed operand form (4 VGPRs for bf16) while it lives across
// phases, instead of the compiler's choice of carrying the f32 values and rounding at the use
__device__ __forceinline__ void pin(frag8& v) {
  typedef unsigned int u32v __attribute__((ext_vector_type(sizeof(frag8) / 4)));
  u32v u = __builtin_bit_cast(u32v, v);
  asm volatile("" : "+v"(u));
  v = __builtin_bit_cast(frag8, u);
}

__device__ __forceinline__ float sum8(const frag8& v) {
#if ASVRL_OPERAND_F32
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) s += static_cast<float>(v[j]);
  return s;
#else
  // four v_dot2_f32_bf16 against ones (exact products, f32 accumulation)
  typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
  const bf16x2 one = {(__bf16)1.0f, (__bf16)1.0f};
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 8; j += 2) s = __builtin_amdgcn_fdot2_f32_bf16(bf16x2{v[j], v[j + 1]}, one, s, false);
  return s;
#endif
}

// MFMA into one of the persistent weight-gradient accumulators, pinned to AGPRs: the other (per-round)
// MFMAs of this file use the VGPR form (built with -mllvm -amdgpu-mfma-vgpr-form=1, build.py), so the
// 256 persistent accumulators fill the AGPR file and the round's working set the VGPR file. The
// accumulators are read only after the round loop, behind mfma_drain().
__device__ __forceinline__ void mfma_acc(f32x16& c, const frag8& a, const frag8& b) {
#if ASVRL_OPERAND_F32
  c = mfma(a, b, c);
#else
  asm("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
#endif
}

// wait states between the last accumulating MFMA (inline asm, invisible to the hazard recognizer)
// and the first VALU read of its result
__device__ __forceinline__ void mfma_drain() {
#if !ASVRL_OPERAND_F32
  asm volatile("s_nop 15\n s_nop 15\n s_nop 15\n s_nop 15" ::: "memory");
#endif
}

// a phase's own lane indices, derived from an opaque copy of threadIdx.x: addresses are then not
// common subexpressions across phases (nor loop invariants of the round loop), whose long live
// ranges would otherwise spill
#define ASVRL_FRESH_LANE()                                        \
  int tid_ = threadIdx.x;                                         \
  asm volatile("" : "+v"(tid_));                                  \
  const int lane = tid_ & 63, h = lane >> 5, r = lane & 31;       \
  (void)h;                                                        \
  (void)r

// Phase timing (tools/fused_stamps.py; a variant build with -DASVRL_FUSED_STAMPS, never the shipped
// library): lane 0 of every wave records s_memtime before and after each of the round's barriers.
#ifdef ASVRL_FUSED_STAMPS
constexpr int kStampRounds = 8, kStamps = 32;   // 0..15: barriers (arrival, release); 16..: marks inside phases
__device__ uint64_t g_stamps[1024 * kNW * kStampRounds * kStamps];
#define ASVRL_STAMP(k)                                                                                   \
  do {                                                                                                   \
    if ((threadIdx.x & 63) == 0 && it_ < kStampRounds && blockIdx.x < 1024)                              \
      g_stamps[((blockIdx.x * kNW + (threadIdx.x >> 6)) * kStampRounds + it_) * kStamps + (k)] =         \
          __builtin_amdgcn_s_memtime();                                                                  \
  } while (0)
#else
#define ASVRL_STAMP(k) \
  do {                 \
  } while (0)
#endif

struct FusedArgs {
  AsvCriticWeights w;
  const float* obs;
  int64_t ld_obs;
  const float* ain;
  int64_t ld_ain;
  void* xb;
  const float* taus;
  const float* qn;
  const float* rew;
  const float* don;
  int64_t ld_rd;
  float gamma, kappa, gscale, loss_scale;
  int B, rounds;
  float* q;
  float* row_loss;
  float* tile_loss;
  void* dzF;
  float* dzG;
  AsvCriticParts parts;
  const float* iwo;   // IQN: output_layer.weight [A][128], bias [A] (f32)
  const float* ibo;
  int n_actions;
  ctile::CriticArgs tq;   // asvrl_critic_train_fused_tq: the target critic's forward (MODE_FWD), q -> qn
};

constexpr int kObsIn = 37;   // self 7 | objects 25 | mask 5 of the packed observation row
constexpr int kEncFloats = 56 * 7 + 56 + 40 * 5 + 40 + 128 * 2 + 128;

// One round's inputs in LDS (floats): obs rows [S][37] | actions [S][NA] | taus [G] | q_next [S][NT] |
// rewards [S] | dones [S]; NA = 2 (AC-IQN's continuous action) or 1 (IQN's action index)
template <int NT, int S, int G, int NA>
struct InLayout {
  static constexpr int kObs = 0, kAct = S * kObsIn, kTau = kAct + NA * S, kQn = kTau + G, kRew = kQn + S * NT,
                       kDon = kRew + S, kSize = kDon + S;
  static constexpr int kPer = (kSize + kNW * 64 - 1) / (kNW * 64);   // elements per thread
};

// Each lane's swizzled-image bases (RowA / TrA of the 64-, 128- and 256-position images), computed once per
// launch into LDS: a phase reads the two or three it uses (ds_read) instead of recomputing them -- about 10
// (RowA) / 25 (TrA) VALU instructions each, ~180 per round, where the round's vector issue, not its matrix work,
// sets its length. Measured 110.2 -> 107.3 us median per launch, bit-identical, SQ_INSTS_VALU -6.3 %
// (profiles/r05k_lane_table_ab.txt; r05_pmc_summary.json). Where the table would not fit beside the images the
// bases are computed.
#ifndef ASVRL_LANE_TABLE
#define ASVRL_LANE_TABLE 1
#endif
// field-major [field][lane]: a phase's reads of one field are 64 consecutive dwords (conflict-free; a lane-major
// table of 12-dword rows put four lanes on each bank)
enum LaneField { kLbR64, kLbR128, kLbR256, kLbT64lo, kLbT64hi, kLbT128lo, kLbT128hi, kLbT256lo, kLbT256hi, kLbFields };
using LaneBases = int[kLbFields][64];
template <int P, bool LT>
__device__ __forceinline__ RowA<P> row_base(const int (*LB)[64], int lane, int r, int h) {
  if constexpr (LT) {
    return RowA<P>(RawBase{}, LB[P == 64 ? kLbR64 : (P == 128 ? kLbR128 : kLbR256)][lane]);
  } else {
    return RowA<P>(r, h);
  }
}
template <int P, bool LT>
__device__ __forceinline__ TrA<P> tr_base(const int (*LB)[64], int lane) {
  if constexpr (LT) {
    constexpr int f = P == 64 ? kLbT64lo : (P == 128 ? kLbT128lo : kLbT256lo);
    return TrA<P>(RawBase{}, LB[f][lane], LB[f + 1][lane]);
  } else {
    return TrA<P>(lane);
  }
}

template <int NT, int NB, int S, bool IQN, int NSB>
struct FusedLds {
  elem_t cos[NSB][32 * NB * kNcos];   // natural order (the cos layer is input-fed); NSB = 2: stage-ahead
  elem_t x[32 * NB * kC];             // F * c
  elem_t a[32 * NB * kH];             // h1g
  elem_t b[32 * NB * kH];             // h2, then dz2 in place
  elem_t dz1[32 * NB * kH];           // IQN: first the one-hot dq image [G][64] (output layer's dZ)
  elem_t dzc[kNW][32 * NB * kNcos];   // each wave's own dzc image (the A operand of its dWc rows)
  float F[NSB][S * kC];               // position order; operand-rounded values held in f32
  float G[NSB][IQN ? 1 : S * kH];     // position order (AC-IQN's action features)
  float qpart[kNW][32 * NB];
  float dq[32 * NB];
  float tsum[2 * NB];                 // loss sums of the round's 16-row groups
  float bias[kC + 3 * kH + 4];        // bc | b1 | b2 | wo, position order | bo
  float woA[IQN ? kMaxA * kH : 4];    // IQN: output_layer.weight, position order, zero rows to 32
  float boA[IQN ? kMaxA : 4];
  float enc[kEncFloats];              // encoder parameters (stage_fg)
  float in[2][InLayout<NT, S, 32 * NB, IQN ? 1 : 2>::kSize];   // the round's inputs, double-buffered
  float red[kNW];
  // AC-IQN with parts.enc / parts.aenc: the encoders' gradient sums over the workgroup's rows, one
  // lane-private slot per (feature, input): [input 0..6 | bias at 7][256 features], natural order;
  // action encoder [w0 | w1 | b][lane half][128 features]
  float encacc[IQN ? 1 : 8 * kC];
  float aeacc[IQN ? 1 : 3 * 2 * kH];
};

constexpr int kSelfF = 56, kSelfIn = 7, kObjF = 40, kObjIn = 5, kObsMask = 32;

// element e of round t's input block (InLayout), read from the kernel's global inputs
template <int NT, int S, int G, int NA>
__device__ __forceinline__ float fetch_in(const FusedArgs& a, int t, int e) {
  // one load from a selected address (a branch per source would serialise the loads)
  using IL = InLayout<NT, S, G, NA>;
  const int64_t b0 = static_cast<int64_t>(t) * S;
  const float* p;
  if (e < IL::kAct) p = a.obs + (b0 + e / kObsIn) * a.ld_obs + e % kObsIn;
  else if (e < IL::kTau) p = a.ain + (b0 + (e - IL::kAct) / NA) * a.ld_ain + (e - IL::kAct) % NA;
  else if (e < IL::kQn) p = a.taus + static_cast<int64_t>(t) * G + (e - IL::kTau);
  else if (e < IL::kRew) p = a.qn + b0 * NT + (e - IL::kQn);
  else if (e < IL::kDon) p = a.rew + (b0 + e - IL::kRew) * a.ld_rd;
  else p = a.don + (b0 + e - IL::kDon) * a.ld_rd;
  return *p;
}

// F (observation_processor, AC_IQN_model.py:284-308) and G (relu(action_encoder(a)),
// AC_IQN_model.py:468-470) of the round's S samples into LDS, position order; xb for the encoder
// weight gradient. f32 dot products in the same order as asvrl_critic.hip's stage_features, from the
// round's staged inputs and the staged encoder parameters.
template <int NT, int S, int G, bool IQN>
__device__ __forceinline__ void stage_fg(const FusedArgs& a, int b0, int tid, const float* in, const float* enc,
                                         float* Fs, float* Gs) {
#pragma clang fp contract(off)
  using IL = InLayout<NT, S, G, IQN ? 1 : 2>;
  constexpr int T = kNW * 64;
  const float* self_w = enc;
  const float* self_b = self_w + 56 * 7;
  const float* obj_w = self_b + 56;
  const float* obj_b = obj_w + 40 * 5;
  const float* ae_w = obj_b + 40;
  const float* ae_b = ae_w + 128 * 2;
  // thread tid: feature m = tid (S * 256 / T samples each); compile-time trip counts, the feature's
  // weights loaded once for all its samples
  static_assert(kC == T, "one cos-layer feature per thread");
  {
    const int m = tid;
    if (m < kSelfF) {
      float w[kSelfIn];
#pragma unroll
      for (int i = 0; i < kSelfIn; ++i) w[i] = self_w[m * kSelfIn + i];
      const float bb = self_b[m];
#pragma unroll
      for (int k = 0; k < S; ++k) {
        const float* x = in + IL::kObs + k * kObsIn;
        float d = 0.f;
#pragma unroll
        for (int i = 0; i < kSelfIn; ++i) d += w[i] * x[i];
        Fs[k * kC + swap23(m)] = static_cast<float>((elem_t)relu(d + bb));
      }
    } else {
      const int o = (m - kSelfF) / kObjF, j = (m - kSelfF) % kObjF;
      float w[kObjIn];
#pragma unroll
      for (int i = 0; i < kObjIn; ++i) w[i] = obj_w[j * kObjIn + i];
      const float bb = obj_b[j];
#pragma unroll
      for (int k = 0; k < S; ++k) {
        const float* x = in + IL::kObs + k * kObsIn;
        const float* xo = x + kSelfIn + kObjIn * o;
        float d = 0.f;
#pragma unroll
        for (int i = 0; i < kObjIn; ++i) d += w[i] * xo[i];
        const float v = x[kObsMask + o] < 0.5f ? 0.f : relu(d + bb);   // masked_fill(mask < 0.5, 0)
        Fs[k * kC + swap23(m)] = static_cast<float>((elem_t)v);        // the operand type's F
      }
    }
  }
  if (!IQN && tid < kH) {
    const int m = tid;
    const float w0 = ae_w[2 * m], w1 = ae_w[2 * m + 1], bb = ae_b[m];
#pragma unroll
    for (int k = 0; k < S; ++k)
      Gs[k * kH + swap23(m)] = relu((w0 * in[IL::kAct + 2 * k] + w1 * in[IL::kAct + 2 * k + 1]) + bb);
  }
  if (a.xb != nullptr && tid < S * 32) {
    const int k = tid / 32, c = tid % 32;
    bp(a.xb)[static_cast<int64_t>(b0 + k) * 32 + c] = (elem_t)in[IL::kObs + k * kObsIn + c];
  }
}

// quantile-Huber terms of one row against its sample's N' = NT targets r + gamma q_next (1 - d)
// (agent.py:399-412), split over four lanes: lane quarter q4 (lanes 16 q4 .. 16 q4 + 15 share the
// row block) takes targets q4 NT/4 .. + NT/4 - 1 (formed once per sample when the round is staged,
// stage_targets), and the four partial sums are combined by two lane exchanges (a fixed order).
// Returns dq; *wl = the row's loss sum.
template <int NT>
__device__ __forceinline__ float quarter_loss_dq(const FusedArgs& a, const float* qt, float tau, float q, int q4,
                                                 float* wl_out) {
  const float kap = a.kappa, hk = 0.5f * a.kappa, omt = 1.f - tau;
  float wl = 0.f, wg = 0.f;
#pragma unroll
  for (int j = 0; j < NT / 4; ++j) {
    const float target = qt[q4 * (NT / 4) + j];
    const float d = target - q;   // td_error (agent.py:406)
    const float ad = fabsf(d);
    const bool quad = ad <= kap;
    const float hub = quad ? 0.5f * (d * d) : kap * (ad - hk);
    const float w = d < 0.f ? omt : tau;
    wl += w * hub;
    wg += w * (quad ? d : copysignf(kap, d));
  }
  // lane-quarter sums on the VALU (v_permlane16/32_swap): the same two-step order as xor shuffles
  // (fp addition of two terms commutes), without two LDS round trips
  wl = half_sum(row_pair_sum(wl));
  wg = half_sum(row_pair_sum(wg));
  *wl_out = wl / kap;
  return -(wg / kap) * a.gscale;
}

// Per-sample sums over the NT rows of each sample (dG, dF) of a wave's 16-feature-per-lane block
// values X[j][g] (row block j, register g, positions base + 16(g>>3) + 8h + (g&7)), by transpose-
// reduce; emit(b_local, position, sum) for every (sample, feature) of the block.
template <int NT, int NB, class Emit>
__device__ __forceinline__ void sample_sums(float (&X)[NB][16], int base, int lane, Emit emit) {
  const int r = lane & 31, h = lane >> 5;
  constexpr int NBR = NT >= 32 ? 2 : 1;
  constexpr int V = 16 * NBR, PER = V / NT;
#pragma unroll
  for (int j0 = 0; j0 < NB; j0 += NBR) {
    float vals[V];
#pragma unroll
    for (int jj = 0; jj < NBR; ++jj)
#pragma unroll
      for (int g = 0; g < 16; ++g) vals[jj * 16 + g] = (j0 + jj < NB) ? X[j0 + jj < NB ? j0 + jj : 0][g] : 0.f;
    xreduce<V, NT>(vals, lane);
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int v = (r % NT) * PER + i, jj = v / 16, g = v % 16;
      if (j0 + jj >= NB) continue;
      const int bl = (32 * (j0 + jj) + (NT >= 32 ? 0 : r)) / NT;
      emit(bl, base + 16 * (g >> 3) + 8 * h + (g & 7), vals[i]);
    }
  }
}

// IQN: the action index of the round's local row lr (clamped as asvrl_critic.hip's IQN_TRAIN)
template <int OFF>
__device__ __forceinline__ int row_action(const float* in, int bl, int A) {
  const int ai = static_cast<int>(in[OFF + bl]);
  return ai < 0 ? 0 : (ai >= A ? A - 1 : ai);
}

// acc[j] += W(ks) B(j, ks) over ks < KS for the NB row blocks, B(j, ks) = rowf(img, RA, j, ks) read D
// k-steps ahead: without the explicit read-ahead and a scheduling fence per k-step the compiler (at its
// VGPR limit) issues each operand read right before its MFMA and waits for it (ds_read, s_waitcnt
// lgkmcnt(0), v_mfma for every MFMA), exposing the LDS latency on every one. Same MFMA order (results
// bit-identical); D = 0: the plain loop. D = 2 (default): round 32.8k -> 28.4k cycles, fused critic
// 125 -> 110.5 us, AC-IQN step 0.316 -> 0.302 ms, IQN 2780 -> 2920 learn-steps/s; D = 3 spills
// (profiles/r02_read_ahead_ab.txt).
#ifndef ASVRL_READ_AHEAD
#define ASVRL_READ_AHEAD 2
#endif
// (Measured in round 4 and removed, profiles/r04e_fused_variants_ab.txt: a deeper weight-gradient read-ahead,
// dW2 + L3 and dW1 + L4 as interleaved MFMA streams, the cos layer's gradient loop a k-step ahead, and the dW2 /
// dW1 partials stored during the last round -- all bit-identical, none faster.)
template <int KS, int NB, int P, class WF>
__device__ __forceinline__ void mfma_rows(f32x16 (&acc)[NB], const elem_t* img, const RowA<P>& RA, WF wf) {
  constexpr int D = ASVRL_READ_AHEAD < KS ? ASVRL_READ_AHEAD : KS;
  if constexpr (D == 0) {
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int j = 0; j < NB; ++j) acc[j] = mfma(wf(ks), rowf(img, RA, j, ks), acc[j]);
  } else {
    frag8 bq[D][NB];
#pragma unroll
    for (int d = 0; d < D; ++d)
#pragma unroll
      for (int j = 0; j < NB; ++j) bq[d][j] = rowf(img, RA, j, d);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
#pragma unroll
      for (int j = 0; j < NB; ++j) acc[j] = mfma(wf(ks), bq[ks % D][j], acc[j]);
      if (ks + D < KS)
#pragma unroll
        for (int j = 0; j < NB; ++j) bq[ks % D][j] = rowf(img, RA, j, ks + D);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
}

// The weight-gradient grid dW[n] += A(kk)^T-read x B(kk, n) over kk < KK, n < NN (mf(kk, n, A, B) does
// the MFMA and, at n = 0, the bias sum): every B(kk, n) read D steps ahead in (kk, n) order, each A(kk)
// a whole kk ahead, one scheduling fence per step (see mfma_rows).
template <int KK, int NN, class AF, class BF, class MF>
__device__ __forceinline__ void mfma_grid(AF af, BF bf, MF mf) {
  constexpr int T = KK * NN, D0 = ASVRL_READ_AHEAD < T ? ASVRL_READ_AHEAD : T;
  if constexpr (D0 == 0) {
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      const frag8 A = af(kk);
#pragma unroll
      for (int n = 0; n < NN; ++n) mf(kk, n, A, bf(kk, n));
    }
  } else {
    constexpr int D = D0;
    frag8 bq[D], aq[2];
    aq[0] = af(0);
#pragma unroll
    for (int t = 0; t < D; ++t) bq[t] = bf(t / NN, t % NN);
#pragma unroll
    for (int t = 0; t < T; ++t) {
      const int kk = t / NN, n = t % NN;
      if (n == 0 && kk + 1 < KK) aq[(kk + 1) % 2] = af(kk + 1);
      mf(kk, n, aq[kk % 2], bq[t % D]);
      if (t + D < T) bq[t % D] = bf((t + D) / NN, (t + D) % NN);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
}

// The target critic's forward in the update's own launch (asvrl_critic_train_fused_tq, and for IQN
// asvrl_iqn_train_fused_tq): before its first round, each workgroup computes q_next for exactly the samples its
// rounds update -- round t's rows are tiles t NB .. t NB + NB - 1 -- with asvrl_critic.hip's forward tile
// (critic_tile<MODE_FWD>, or <MODE_IQN_MAX> for IQN's max over the actions: the same code and arithmetic,
// bit-identical q_next), the target weights staged in the LDS the rounds use afterwards, then stores them where
// the rounds' input fetch reads q_next (global, workgroup-coherent after the barrier). No workgroup waits on
// another: the samples of different workgroups are disjoint.
template <int NT, bool TQ, bool IQN> struct TqLds { float pad[4]; };
// N = 32 (a tile = one sample): the workgroup's samples are staged 16 at a time by all its threads together
// (F, G and the taus of the chunk's tiles), so the tiles then run without a global load
constexpr int kTqChunk = 16;
template <int NT, bool IQN> struct TqLds<NT, true, IQN> {
  using FT = typename ctile::FOf<IQN ? ctile::MODE_IQN_MAX : ctile::MODE_FWD>::T;   // the tile's F element
  using WT = typename ctile::LdsOf<IQN ? ctile::MODE_IQN_MAX : ctile::MODE_FWD>::T;
  static constexpr int kF = NT == 32 ? kTqChunk * kC : kNW * (32 / NT) * kC;
  static constexpr int kG = IQN ? 4 : (NT == 32 ? kTqChunk * kH : kNW * (32 / NT) * kH);   // IQN: no action features
  WT W;
  FT F[kF];
  float G[kG];
  float T[NT == 32 ? kTqChunk * 32 : 4];
};
template <int NT, int NB, int S, bool IQN, int NSB, bool TQ>
union FusedShared {
  FusedLds<NT, NB, S, IQN, NSB> f;
  TqLds<NT, TQ, IQN> t;
};

// F, G (asvrl_critic_tile.h stage_features' arithmetic, op for op, uncontracted) and the taus of n <= 16
// samples b(0..n-1): thread m computes feature m of every sample from its weights loaded once. WITH_G false
// (IQN): no action features.
template <bool WITH_G, class FT, class BF>
__device__ __forceinline__ void tq_stage_chunk(const ctile::CriticArgs& t, int n, BF bidx, FT* F, float* G,
                                               float* T) {
#pragma clang fp contract(off)
  const int m = threadIdx.x;   // kNW * 64 == kC threads: one feature each
  static_assert(kNW * 64 == kC, "one thread per feature");
  const bool self = m < ctile::kSelfF;
  const int o = self ? 0 : (m - ctile::kSelfF) / ctile::kObjF, j = self ? 0 : (m - ctile::kSelfF) % ctile::kObjF;
  const float* wp = self ? t.w.self_w + m * ctile::kSelfIn : t.w.obj_w + j * ctile::kObjIn;
  float w[ctile::kSelfIn];
#pragma unroll
  for (int i = 0; i < ctile::kSelfIn; ++i) w[i] = wp[(i < ctile::kObjIn || self) ? i : 0];
  const float bb = self ? t.w.self_b[m] : t.w.obj_b[j];
  const int xo = self ? 0 : ctile::kSelfIn + ctile::kObjIn * o;
  float ae0 = 0.f, ae1 = 0.f, aeb = 0.f;
  if (WITH_G && m < kH) {
    ae0 = t.w.ae_w[2 * m];
    ae1 = t.w.ae_w[2 * m + 1];
    aeb = t.w.ae_b[m];
  }
  constexpr int kSub = 8;   // samples whose loads are in flight together (register budget)
  for (int k0 = 0; k0 < n; k0 += kSub) {
    float xs[kSub][ctile::kSelfIn], mk[kSub], a0[kSub], a1[kSub], tv[kSub];
#pragma unroll
    for (int q = 0; q < kSub; ++q) {   // every load of the batch issued before the first use
      const int k = k0 + q;
      const int b = k < n ? bidx(k) : bidx(k0);
      const float* x = t.obs + static_cast<int64_t>(b) * t.ld_obs;
#pragma unroll
      for (int i = 0; i < ctile::kSelfIn; ++i) xs[q][i] = x[xo + ((i < ctile::kObjIn || self) ? i : 0)];
      mk[q] = self ? 1.f : x[ctile::kObsMask + o];
      a0[q] = WITH_G ? t.ain[static_cast<int64_t>(b) * t.ld_ain] : 0.f;
      a1[q] = WITH_G ? t.ain[static_cast<int64_t>(b) * t.ld_ain + 1] : 0.f;
      tv[q] = t.taus[static_cast<int64_t>(b) * 32 + (m & 31)];   // NT = 32: tile b's rows
    }
#pragma unroll
    for (int q = 0; q < kSub; ++q) {
      const int k = k0 + q;
      if (k >= n) break;
      float d = 0.f;
#pragma unroll
      for (int i = 0; i < ctile::kSelfIn; ++i)
        if (i < ctile::kObjIn || self) d += w[i] * xs[q][i];
      const float v = mk[q] < 0.5f ? 0.f : relu(d + bb);   // masked_fill(mask < 0.5, 0)
      F[k * kC + m] = static_cast<FT>((elem_t)v);
      if (WITH_G && m < kH) G[k * kH + m] = relu((ae0 * a0[q] + ae1 * a1[q]) + aeb);
      if (m < 32) T[k * 32 + m] = tv[q];
    }
  }
}

template <int NT, int NB, bool IQN>
__device__ __forceinline__ void target_phase(const ctile::CriticArgs& t, TqLds<NT, true, IQN>& T, int rounds) {
  constexpr int MODE = IQN ? ctile::MODE_IQN_MAX : ctile::MODE_FWD;
  constexpr int St = 32 / NT;
  const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // N = 32: the Wc and W2 images' fragments (8 + 8 per thread) are loaded into registers first and stored to
  // LDS after the first chunk of samples is staged, so their L2 round trip runs under the chunk's own loads
  constexpr bool kEarly = kWeightsInLds && NT == 32;
  constexpr int kPerC = ctile::kFragWC / (kNW * 64), kPer2 = ctile::kFragW2 / (kNW * 64);
  static_assert(!kEarly || (kPerC * kNW * 64 == ctile::kFragWC && kPer2 * kNW * 64 == ctile::kFragW2), "whole images");
  frag8 ec[kEarly ? kPerC : 1], e2[kEarly ? kPer2 : 1];
  if constexpr (kEarly) {
#pragma unroll
    for (int c = 0; c < kPerC; ++c) ec[c] = reinterpret_cast<const frag8*>(t.w.wc_frag)[c * kNW * 64 + threadIdx.x];
#pragma unroll
    for (int c = 0; c < kPer2; ++c) e2[c] = reinterpret_cast<const frag8*>(t.w.w2_frag)[c * kNW * 64 + threadIdx.x];
    copy_frags<kNW * 64, ctile::kFragW1, 16>(T.W.w1, reinterpret_cast<const frag8*>(t.w.w1_frag), threadIdx.x);
  } else if constexpr (kWeightsInLds) {
    copy_frags<kNW * 64, ctile::kFragWC, 16>(T.W.wc, reinterpret_cast<const frag8*>(t.w.wc_frag), threadIdx.x);
    copy_frags<kNW * 64, ctile::kFragW1, 16>(T.W.w1, reinterpret_cast<const frag8*>(t.w.w1_frag), threadIdx.x);
    copy_frags<kNW * 64, ctile::kFragW2, 16>(T.W.w2, reinterpret_cast<const frag8*>(t.w.w2_frag), threadIdx.x);
  }
  for (int i = threadIdx.x; i < kC; i += kNW * 64) T.W.bc[i] = t.w.bc[i];
  for (int i = threadIdx.x; i < kH; i += kNW * 64) {
    T.W.b1[i] = t.w.b1[i];
    T.W.b2[i] = t.w.b2[i];
    if constexpr (!IQN) T.W.wo[i] = t.w.wo[i];
  }
  if constexpr (IQN) {   // the head image and its bias (critic_kernel's staging for the IQN modes)
    const frag8* gwo = reinterpret_cast<const frag8*>(t.hd.wo_frag);
    for (int i = threadIdx.x; i < kH / 16 * 64; i += kNW * 64) T.W.wo_img[i] = gwo[i];
    for (int i = threadIdx.x; i < kMaxA; i += kNW * 64) T.W.bo_a[i] = i < t.hd.n_actions ? t.hd.bo[i] : 0.f;
  }
  const int mine = (rounds - static_cast<int>(blockIdx.x) + static_cast<int>(gridDim.x) - 1) / static_cast<int>(gridDim.x) * NB;
  auto tile_of = [&](int i) { return (static_cast<int>(blockIdx.x) + (i / NB) * static_cast<int>(gridDim.x)) * NB + i % NB; };
  if constexpr (NT == 32) {
#pragma nounroll
    for (int c0 = 0; c0 < mine; c0 += kTqChunk) {   // workgroup-uniform
      const int n = mine - c0 < kTqChunk ? mine - c0 : kTqChunk;
      tq_stage_chunk<!IQN>(t, n, [&](int k) { return tile_of(c0 + k); }, T.F, T.G, T.T);
      if constexpr (kEarly) {
        if (c0 == 0) {
#pragma unroll
          for (int c = 0; c < kPerC; ++c) T.W.wc[c * kNW * 64 + threadIdx.x] = ec[c];
#pragma unroll
          for (int c = 0; c < kPer2; ++c) T.W.w2[c * kNW * 64 + threadIdx.x] = e2[c];
        }
      }
      __syncthreads();
#pragma nounroll
      for (int k = wv; k < n; k += kNW)
      {
        int kk = k;   // opaque VGPR copy: with a uniform k the tile's LDS addresses are hoisted and spill (573)
        asm volatile("" : "+v"(kk));
        ctile::critic_tile<MODE, NT>(t, T.W, tile_of(c0 + kk), lane, T.F + kk * kC, IQN ? nullptr : T.G + kk * kH,
                                     nullptr, T.T + kk * 32);
      }
      __syncthreads();
    }
  } else {
    __syncthreads();
    auto* Fw = T.F + wv * St * kC;
    float* Gw = IQN ? nullptr : T.G + wv * St * kH;
    for (int i = wv; i < mine; i += kNW) {
      const int tile = tile_of(i);
      ctile::stage_features<NT, !IQN, false>(t, tile, lane, Fw, Gw);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");   // the wave's own rows: in-order LDS, compiler fence
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      ctile::critic_tile<MODE, NT>(t, T.W, tile, lane, Fw, Gw);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    __syncthreads();   // every q_next of the workgroup stored; the LDS is the update's from here
  }
}


template <int NT, bool IQN, bool TQ = false>
__global__ __launch_bounds__(kNW * 64) __attribute__((amdgpu_waves_per_eu(1, 1)))
void critic_fused_kernel(FusedArgs a) {
  constexpr int NB = FusedNB<NT>::v, G = 32 * NB, S = G / NT, NA = IQN ? 1 : 2;
  constexpr bool AH = ASVRL_STAGE_AHEAD && (!IQN || ASVRL_STAGE_AHEAD_IQN) && NT == 32 && !ASVRL_OPERAND_F32;
  constexpr int NSB = AH ? 2 : 1;
  __shared__ __attribute__((aligned(16))) FusedShared<NT, NB, S, IQN, NSB, TQ> U;
  static_assert(sizeof(U) <= 160 * 1024, "fused critic LDS image exceeds the CU's 160 KB");
  constexpr bool LT = ASVRL_LANE_TABLE && sizeof(U) + sizeof(LaneBases) <= 160 * 1024;
  __shared__ int LB[LT ? kLbFields : 1][64];   // each lane's image bases
  auto& L = U.f;
  if constexpr (TQ) target_phase<NT, NB, IQN>(a.tq, U.t, a.rounds);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 5, r = lane & 31;
  if constexpr (LT) {   // read after the prologue's barrier
    if (threadIdx.x < 64) {
      // the constructors themselves (row_base / tr_base read this table)
      LB[kLbR64][lane] = RowA<kNcos>(r, h).base;
      LB[kLbR128][lane] = RowA<kH>(r, h).base;
      LB[kLbR256][lane] = RowA<kC>(r, h).base;
      const auto t64 = TrA<kNcos>(lane);
      const auto t128 = TrA<kH>(lane);
      const auto t256 = TrA<kC>(lane);
      LB[kLbT64lo][lane] = t64.lo;
      LB[kLbT64hi][lane] = t64.hi;
      LB[kLbT128lo][lane] = t128.lo;
      LB[kLbT128hi][lane] = t128.hi;
      LB[kLbT256lo][lane] = t256.lo;
      LB[kLbT256hi][lane] = t256.hi;
    }
  }
  const frag8* WC = reinterpret_cast<const frag8*>(a.w.wc_frag);
  const frag8* W1 = reinterpret_cast<const frag8*>(a.w.w1_frag);
  const frag8* W2 = reinterpret_cast<const frag8*>(a.w.w2_frag);
  const frag8* W2T = reinterpret_cast<const frag8*>(a.w.w2t_frag);
  const frag8* W1T = reinterpret_cast<const frag8*>(a.w.w1t_frag);
  float* const bcp = L.bias;
  float* const b1p = L.bias + kC;
  float* const b2p = L.bias + kC + kH;
  float* const wop = L.bias + kC + 2 * kH;
  for (int i = threadIdx.x; i < kC; i += kNW * 64) bcp[swap23(i)] = a.w.bc[i];
  for (int i = threadIdx.x; i < kH; i += kNW * 64) {
    b1p[swap23(i)] = a.w.b1[i];
    b2p[swap23(i)] = a.w.b2[i];
    if constexpr (!IQN) wop[swap23(i)] = a.w.wo[i];
  }
  if constexpr (IQN) {   // the head, rows >= n_actions zero (never gathered: actions are clamped)
    for (int i = threadIdx.x; i < kMaxA * kH; i += kNW * 64) {
      const int row = i / kH, col = i % kH;
      L.woA[row * kH + swap23(col)] = row < a.n_actions ? a.iwo[i] : 0.f;
    }
    if (threadIdx.x < kMaxA) L.boA[threadIdx.x] = threadIdx.x < a.n_actions ? a.ibo[threadIdx.x] : 0.f;
  } else {
    if (threadIdx.x == 0) L.bias[kC + 3 * kH] = a.w.bo[0];
  }

  using IL = InLayout<NT, S, G, NA>;
  {
    // the encoder parameters into LDS: each thread's (at most five) loads issued before its stores
    constexpr int kEncN = IQN ? 56 * 7 + 56 + 40 * 5 + 40 : kEncFloats, kEncPer = (kEncN + kNW * 64 - 1) / (kNW * 64);
    float ev[kEncPer];
#pragma unroll
    for (int u = 0; u < kEncPer; ++u) {
      int e = threadIdx.x + u * kNW * 64;
      const float* src = a.w.self_w;
      if (e >= 392) { e -= 392; src = a.w.self_b;
        if (e >= 56) { e -= 56; src = a.w.obj_w;
          if (e >= 200) { e -= 200; src = a.w.obj_b;
            if (e >= 40) { e -= 40; src = a.w.ae_w;
              if (e >= 256) { e -= 256; src = a.w.ae_b; } } } } }
      ev[u] = threadIdx.x + u * kNW * 64 < kEncN ? src[e] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < kEncPer; ++u)
      if (threadIdx.x + u * kNW * 64 < kEncN) L.enc[threadIdx.x + u * kNW * 64] = ev[u];
    if constexpr (!IQN) {
      for (int i = threadIdx.x; i < 8 * kC; i += kNW * 64) L.encacc[i] = 0.f;
      for (int i = threadIdx.x; i < 3 * 2 * kH; i += kNW * 64) L.aeacc[i] = 0.f;
    }
    if (blockIdx.x < a.rounds)
#pragma unroll
      for (int u = 0; u < IL::kPer; ++u) {
        const int e = threadIdx.x + u * kNW * 64;
        if (e < IL::kSize) L.in[0][e] = fetch_in<NT, S, G, NA>(a, blockIdx.x, e);
      }
  }
  __syncthreads();

  // one round's F, G, xb (stage_fg) and cos(tau pi k) rows (natural order) from its staged inputs
  auto stage = [&](int b0s, float* ins, elem_t* cosd, float* Fd, float* Gd) {
    int tid_s = threadIdx.x;
    asm volatile("" : "+v"(tid_s));
    stage_fg<NT, S, G, IQN>(a, b0s, tid_s, ins, L.enc, Fd, Gd);
    // the round's quantile targets r + gamma q_next (1 - d) (agent.py:399-400), once per (sample, j)
    // in place over q_next, instead of in every row's loss terms
    static_assert(S * NT <= kNW * 64, "one target per thread");
    if (tid_s < S * NT) {
      const int k = tid_s / NT;
      float* qn = ins + IL::kQn + tid_s;
      *qn = ins[IL::kRew + k] + (a.gamma * *qn) * (1.0f - ins[IL::kDon + k]);
    }
    static_assert((G * (kNcos / 8)) % (kNW * 64) == 0, "whole cos chunks per thread");
#pragma unroll
    for (int u = 0; u < G * (kNcos / 8) / (kNW * 64); ++u) {
      const int c = tid_s + u * kNW * 64;
      const int row = c / (kNcos / 8), ch = c % (kNcos / 8);
      const float tau = ins[IL::kTau + row];
      float cv[8];
      cos_pi_k_tau8r(tau, 8 * ch, cv);
      row_store<kNcos>(cosd, row, 8 * ch, pack8(cv));
    }
  };
  if constexpr (AH) {
    if (blockIdx.x < a.rounds) stage(blockIdx.x * G / NT, L.in[0], L.cos[0], L.F[0], L.G[0]);
    __syncthreads();
  }

  // persistent per-wave weight-gradient accumulators (rows = this wave's features, positions)
  f32x16 dW2[4], dW1[8], dWc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) dW2[i] = dWc[i] = f32x16{};
#pragma unroll
  for (int i = 0; i < 8; ++i) dW1[i] = f32x16{};
  float db2 = 0.f, db1 = 0.f, dbc0 = 0.f, dbc1 = 0.f, dbo = 0.f;
  // output layer: AC-IQN's single row (per-lane sums over rows), IQN's [32 actions][own 32 features]
  // MFMA block (rows = actions)
  float dwo[IQN ? 1 : 16];
  f32x16 dWo = f32x16{};
#pragma unroll
  for (int g = 0; g < (IQN ? 1 : 16); ++g) dwo[g] = 0.f;
  constexpr bool WCR = AH && ASVRL_WC_RESIDENT;
  frag8 wcr0[WCR ? 4 : 1], wcr1[WCR ? 4 : 1];   // resident cos-layer fragments (blocks 2w, 2w + 1)
  if constexpr (WCR) {
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      wcr0[ks] = WC[((2 * w) * 4 + ks) * 64 + lane];
      wcr1[ks] = WC[((2 * w + 1) * 4 + ks) * 64 + lane];
    }
  }
  float encr[IQN ? 8 : 1];   // IQN with parts.enc: this lane's feature's encoder sums
#pragma unroll
  for (int i = 0; i < (IQN ? 8 : 1); ++i) encr[i] = 0.f;
  const int grp = blockIdx.x;
  int buf = 0, it_ = 0;
  (void)it_;
  for (int t = blockIdx.x; t < a.rounds; t += gridDim.x, buf ^= 1, ++it_) {
    // the next round's inputs, into registers during this round and into LDS at its end
    float pre[IL::kPer];
    int tid_p = threadIdx.x;
    asm volatile("" : "+v"(tid_p));
#define ASVRL_FETCH_PRE()                                                                   \
  _Pragma("unroll") for (int u = 0; u < IL::kPer; ++u) {                                   \
    const int e = tid_p + u * kNW * 64;                                                    \
    pre[u] = (t + static_cast<int>(gridDim.x) < a.rounds && e < IL::kSize)                 \
                 ? fetch_in<NT, S, G, NA>(a, t + gridDim.x, e) : 0.f;                      \
  }
    float* const in = L.in[buf];
    // the lane indices re-derived through an opaque copy every round: otherwise every LDS / weight
    // address of the round body is loop-invariant, gets hoisted out of the loop and spills
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int row0 = t * G, b0 = row0 / NT;
    elem_t* const dzc_w = L.dzc[w];
    // ---------------- stage: F, G, xb; cos(tau pi k) for the round's rows (natural order); the
    // cos layer's weight fragments are fetched meanwhile
    frag8 wc0[4], wc1[4];
    if constexpr (WCR) {
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        wc0[ks] = wcr0[ks];
        wc1[ks] = wcr1[ks];
      }
    } else {
      ASVRL_FRESH_LANE();
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        wc0[ks] = WC[((2 * w) * 4 + ks) * 64 + lane];
        wc1[ks] = WC[((2 * w + 1) * 4 + ks) * 64 + lane];
      }
    }
    const int sb = AH ? buf : 0;   // this round's F, G, cos images
    elem_t* const cosb = L.cos[sb];
    float* const Fb = L.F[sb];
    float* const Gb = L.G[sb];
    if constexpr (!AH) {
      stage(b0, in, cosb, Fb, Gb);
      ASVRL_STAMP(0);
      __syncthreads();
      ASVRL_STAMP(1);
    } else {   // staged by the previous round (or the prologue)
      ASVRL_STAMP(0);
      ASVRL_STAMP(1);
    }

    // ---------------- L0: c = relu(Wc cos + bc), x = F * c      (this wave: blocks 2w, 2w+1); W1 fetched
    frag8 w1f[16];
    {
      ASVRL_FRESH_LANE();
      const RowA<kNcos> RA_cos = row_base<kNcos, LT>(LB, lane, r, h);
      const RowA<kC> RA_x = row_base<kC, LT>(LB, lane, r, h);
      // the cos rows' operand fragments are the same for both blocks: with read-ahead, all read first
      frag8 cb[ASVRL_READ_AHEAD ? NB : 1][4];
      if constexpr (ASVRL_READ_AHEAD != 0) {
#pragma unroll
        for (int j = 0; j < NB; ++j)
#pragma unroll
          for (int ks = 0; ks < 4; ++ks) cb[j][ks] = rowf(cosb, RA_cos, j, ks);
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int mq = 0; mq < 2; ++mq) {
        const int mb = 2 * w + mq;
        float fv[NB][2][8];
#pragma unroll
        for (int j = 0; j < NB; ++j)
#pragma unroll
          for (int s = 0; s < 2; ++s) lds8(Fb + ((32 * j + r) / NT) * kC + mb * 32 + 16 * s + 8 * h, fv[j][s]);
#pragma unroll
        for (int j = 0; j < NB; ++j) {
          f32x16 acc = acc_init(bcp, mb * 32, h);
#pragma unroll
          for (int ks = 0; ks < 4; ++ks)
            acc = mfma(mq ? wc1[ks] : wc0[ks], ASVRL_READ_AHEAD ? cb[ASVRL_READ_AHEAD ? j : 0][ks]
                                                                  : rowf(cosb, RA_cos, j, ks), acc);
          if constexpr (!kBiasFirst) acc += bias_init(bcp, mb * 32, h);
#pragma unroll
          for (int s = 0; s < 2; ++s) {
            // F >= 0 (a ReLU output), so round(F relu(c)) = relu(round(F c)) up to the sign of a zero:
            // the ReLU on the packed product (v_pk_max_i16, two values per instruction)
            float cv[8], xv[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) cv[i] = acc[8 * s + i];
            mul8(fv[j][s], cv, xv);
            rows(L.x, RA_x, j, 2 * mb + s, relu_packed(pack8(xv)));
          }
        }
        if (mq == 0) ASVRL_STAMP(16);
      }
#pragma unroll
      for (int ks = 0; ks < kC / 16; ++ks) w1f[ks] = W1[(w * 16 + ks) * 64 + lane];
    }
    ASVRL_STAMP(2);
    __syncthreads();
    ASVRL_STAMP(3);

    // ---------------- L1: h1 = relu(W1 x + b1) (own block w), h1g = h1 * G; W2 fetched
    frag8 h1k[NB][2];
    frag8 w2f[8];
    {
      ASVRL_FRESH_LANE();
      const RowA<kC> RA_x = row_base<kC, LT>(LB, lane, r, h);
      const RowA<kH> RA_a = row_base<kH, LT>(LB, lane, r, h);
      float gv[NB][2][8];
      if constexpr (!IQN)
#pragma unroll
        for (int j = 0; j < NB; ++j)
#pragma unroll
          for (int s = 0; s < 2; ++s) lds8(Gb + ((32 * j + r) / NT) * kH + w * 32 + 16 * s + 8 * h, gv[j][s]);
      f32x16 acc[NB];
#pragma unroll
      for (int j = 0; j < NB; ++j) acc[j] = acc_init(b1p, w * 32, h);
      mfma_rows<kC / 16, NB>(acc, L.x, RA_x, [&](int ks) { return w1f[ks]; });
      ASVRL_STAMP(17);
#pragma unroll
      for (int ks = 0; ks < 8; ++ks) w2f[ks] = W2[(w * 8 + ks) * 64 + lane];
      // issued behind W2's fragments: the wait for those (in L2) does not include this load, whose
      // first waiter (W2^T's fragments, in L3) comes two phases later
      ASVRL_FETCH_PRE();
      if constexpr (!kBiasFirst)
#pragma unroll
        for (int j = 0; j < NB; ++j) acc[j] += bias_init(b1p, w * 32, h);
#pragma unroll
      for (int j = 0; j < NB; ++j) {
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          float hv[8], gov[8];
#pragma unroll
          for (int i = 0; i < 8; ++i) hv[i] = relu(acc[j][8 * s + i]);
          h1k[j][s] = pack8(hv);
          if constexpr (!IQN) mul8(hv, gv[j][s], gov);
          rows(L.a, RA_a, j, 2 * w + s, IQN ? h1k[j][s] : pack8(gov));
          pin(h1k[j][s]);
        }
      }
    }
    ASVRL_STAMP(4);
    __syncthreads();
    ASVRL_STAMP(5);

    // ---------------- L2: z2 = W2 h1g + b2 (own block w); partial q over its 32 features; h2 = relu(z2)
    // parked in the dz2 image (operand type) until dq is known; W2^T fetched
    frag8 w2tf[8];
    {
      ASVRL_FRESH_LANE();
      const RowA<kH> RA_a = row_base<kH, LT>(LB, lane, r, h);
      const RowA<kH> RA_b = row_base<kH, LT>(LB, lane, r, h);
      f32x16 z2[NB];
#pragma unroll
      for (int j = 0; j < NB; ++j) z2[j] = acc_init(b2p, w * 32, h);
      mfma_rows<kH / 16, NB>(z2, L.a, RA_a, [&](int ks) { return w2f[ks]; });
      ASVRL_STAMP(18);
#pragma unroll
      for (int ks = 0; ks < 8; ++ks) w2tf[ks] = W2T[(w * 8 + ks) * 64 + lane];
      if constexpr (!kBiasFirst)
#pragma unroll
        for (int j = 0; j < NB; ++j) z2[j] += bias_init(b2p, w * 32, h);
      // the output row feeding q: AC-IQN's single row, IQN's row of the sample's action
      constexpr int NWO = IQN ? NB : 1;
      float wov[NWO][2][8];
#pragma unroll
      for (int j = 0; j < NWO; ++j) {
        const float* src = IQN ? L.woA + row_action<IL::kAct>(in, (32 * j + r) / NT, a.n_actions) * kH : wop;
#pragma unroll
        for (int s = 0; s < 2; ++s) lds8(src + w * 32 + 16 * s + 8 * h, wov[j][s]);
      }
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        float part = 0.f;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          float hv[8];
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const float h2 = relu(z2[j][8 * s + i]);
            part += wov[IQN ? j : 0][s][i] * h2;
            hv[i] = h2;
          }
          rows(L.b, RA_b, j, 2 * w + s, pack8(hv));
        }
        part = half_sum(part);
        if (h == 0) L.qpart[w][32 * j + r] = part;
      }
    }
    ASVRL_STAMP(6);
    __syncthreads();
    ASVRL_STAMP(7);

    // ---------------- loss: q = sum of the four partials + bo; quantile-Huber -> dq. Every wave takes
    // 16-row groups (rows 16 g + (lane & 15)), each row's targets split over the four lane quarters
    {
      ASVRL_FRESH_LANE();
      const int q4 = lane >> 4;
      for (int g = w; g < G / 16; g += kNW) {
        const int lr = 16 * g + (lane & 15), grow = row0 + lr, b = grow / NT;
        const int bl = b - b0;
        int ai = 0;
        if constexpr (IQN) ai = row_action<IL::kAct>(in, bl, a.n_actions);
        const float bo = IQN ? L.boA[ai] : L.bias[kC + 3 * kH];
        const float q = (((L.qpart[0][lr] + L.qpart[1][lr]) + L.qpart[2][lr]) + L.qpart[3][lr]) + bo;
        float wl;
        const float dq = quarter_loss_dq<NT>(a, in + IL::kQn + bl * NT, in[IL::kTau + lr], q, q4, &wl);
        if (a.tile_loss != nullptr) {
          const float v = seg_sum<16>(wl);   // every lane of the 16-lane row: the group's sum
          if (lane == 0) L.tsum[g] = v;
        }
        if (q4 == 0) {
          L.dq[lr] = dq;
          if (a.row_loss != nullptr) a.row_loss[grow] = wl;
          if (a.q != nullptr) a.q[grow] = q;
          if constexpr (!IQN) dbo += dq;
        }
        if constexpr (IQN) {   // the output layer's dZ row: dq at the taken action (agent.py:456 gather)
          frag8 o;
#pragma unroll
          for (int i = 0; i < 8; ++i) o[i] = (elem_t)(8 * q4 + i == ai ? dq : 0.f);
          row_store<64>(L.dz1, lr, 8 * q4, o);
        }
      }
      ASVRL_STAMP(31);
    }
    ASVRL_STAMP(8);
    __syncthreads();
    ASVRL_STAMP(9);

    // ---------------- dz2 = dq wo 1[h2 > 0] (own block, in place over h2), output layer's gradient
    // sum of dq h2; the loss partial of each 32-row tile from its two 16-row sums
    if (a.tile_loss != nullptr && threadIdx.x < G / 32)
      a.tile_loss[row0 / 32 + threadIdx.x] = (L.tsum[2 * threadIdx.x] + L.tsum[2 * threadIdx.x + 1]) * a.loss_scale;
    {
      ASVRL_FRESH_LANE();
      const RowA<kH> RA_b = row_base<kH, LT>(LB, lane, r, h);
      if constexpr (IQN) {
        // dW_out[:, own] += D^T h2 with D the one-hot dq image (rows = actions): h2 read before the
        // in-place dz2 stores below (same wave, in-order LDS)
        const TrA<64> TA_o = tr_base<64, LT>(LB, lane);
        const TrA<kH> TA_b = tr_base<kH, LT>(LB, lane);
#pragma unroll
        for (int kk = 0; kk < G / 16; ++kk) {
          const frag8 A = trf(L.dz1, TA_o, kk, 0);
          dbo += sum8(A);
          dWo = mfma(A, trf(L.b, TA_b, kk, w), dWo);
        }
      }
      // every LDS operand first (one wait), then the arithmetic and the in-place stores
      constexpr int NWO = IQN ? NB : 1;
      float wov[NWO][2][8], dqv[NB];
      frag8 hv[NB][2];
#pragma unroll
      for (int j = 0; j < NWO; ++j) {
        const float* src = IQN ? L.woA + row_action<IL::kAct>(in, (32 * j + r) / NT, a.n_actions) * kH : wop;
#pragma unroll
        for (int s = 0; s < 2; ++s) lds8(src + w * 32 + 16 * s + 8 * h, wov[j][s]);
      }
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        dqv[j] = L.dq[32 * j + r];
#pragma unroll
        for (int s = 0; s < 2; ++s) hv[j][s] = rowf(L.b, RA_b, j, 2 * w + s);
      }
#pragma unroll
      for (int j = 0; j < NB; ++j) {
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          float dz[8];
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            dz[i] = dqv[j] * wov[IQN ? j : 0][s][i];
            if constexpr (!IQN) dwo[8 * s + i] += dqv[j] * static_cast<float>(hv[j][s][i]);
          }
          rows(L.b, RA_b, j, 2 * w + s, mask_pos(pack8(dz), hv[j][s]));   // dq wo 1[h2 > 0]
        }
      }
    }
    ASVRL_STAMP(10);
    __syncthreads();
    ASVRL_STAMP(11);

    // ---------------- dW2[own][:] += dz2^T h1g;  L3: dh1g = W2^T dz2 (own block) -> dG, dz1 (own
    // slice into the dz1 image, which nobody reads before the next barrier)
    {
      ASVRL_FRESH_LANE();
      const TrA<kH> TA_a = tr_base<kH, LT>(LB, lane);
      const TrA<kH> TA_b = tr_base<kH, LT>(LB, lane);
      mfma_grid<G / 16, 4>([&](int kk) { return trf(L.b, TA_b, kk, w); },
                           [&](int kk, int n) { return trf(L.a, TA_a, kk, n); },
                           [&](int kk, int n, const frag8& A, const frag8& B) {
                             if (n == 0) db2 += sum8(A);
                             mfma_acc(dW2[n], A, B);
                           });
      ASVRL_STAMP(19);
    }
    {
      ASVRL_FRESH_LANE();
      const RowA<kH> RA_b = row_base<kH, LT>(LB, lane, r, h);
      const RowA<kH> RA_d = row_base<kH, LT>(LB, lane, r, h);
      float gv[NB][2][8];
      if constexpr (!IQN)
#pragma unroll
        for (int j = 0; j < NB; ++j)
#pragma unroll
          for (int s = 0; s < 2; ++s) lds8(Gb + ((32 * j + r) / NT) * kH + w * 32 + 16 * s + 8 * h, gv[j][s]);
      f32x16 acc[NB];
#pragma unroll
      for (int j = 0; j < NB; ++j) acc[j] = f32x16{};
      mfma_rows<kH / 16, NB>(acc, L.b, RA_b, [&](int ks) { return w2tf[ks]; });
      ASVRL_STAMP(20);
      // dz1 = dh1g G 1[h1 > 0]; dG = sum over the sample's taus of dh1g h1 (-> dzG = dG 1[G > 0])
#pragma unroll
      for (int j = 0; j < NB; ++j) {   // h1 unpacked here, not earlier
        pin(h1k[j][0]);
        pin(h1k[j][1]);
      }
      float gsa[NB][16];
#pragma unroll
      for (int j = 0; j < NB; ++j) {
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          float h1[8], d[8], dg[8], hd[8], dz1[8];
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            h1[i] = static_cast<float>(h1k[j][s][i]);
            d[i] = acc[j][8 * s + i];
          }
          if constexpr (!IQN) mul8(d, gv[j][s], dg);
          mul8(d, h1, hd);
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            dz1[i] = IQN ? d[i] : dg[i];
            gsa[j][8 * s + i] = hd[i];
          }
          rows(L.dz1, RA_d, j, 2 * w + s, mask_pos(pack8(dz1), h1k[j][s]));   // 1[h1 > 0]
        }
      }
      ASVRL_STAMP(21);
      if constexpr (!IQN) {
        const bool enc = a.parts.aenc != nullptr;
        sample_sums<NT, NB>(gsa, w * 32, lane, [&](int bl, int p, float v) {
          const float gm = Gb[bl * kH + p];
          const float dz = gm > 0.f ? v : 0.f;
          if (a.dzG != nullptr) a.dzG[static_cast<size_t>(b0 + bl) * kH + swap23(p)] = dz;
          if (enc) Gb[bl * kH + p] = dz;   // G's block w is this wave's own: dzG in place
        });
        if (enc) {
          // action_encoder's gradient (AC_IQN_model.py:468-470): lane (half hh, position 32w + rr)
          // sums dzG[b] * (a_b0, a_b1, 1) over its half of the round's samples, in sample order
          const int hh = lane >> 5, rr = lane & 31, p = w * 32 + rr, m = swap23(p);
          float s0 = 0.f, s1 = 0.f, sb = 0.f;
#pragma unroll
          for (int k = hh; k < S; k += 2) {
            const float d = Gb[k * kH + p];
            s0 += d * in[IL::kAct + 2 * k];
            s1 += d * in[IL::kAct + 2 * k + 1];
            sb += d;
          }
          float* acc = L.aeacc + hh * kH + m;
          acc[0] += s0;
          acc[2 * kH] += s1;
          acc[4 * kH] += sb;
        }
      }
    }
    if constexpr (AH) {   // the next round's inputs, for its staging in this round's last phase
#pragma unroll
      for (int u = 0; u < IL::kPer; ++u) {
        const int e = tid_p + u * kNW * 64;
        if (e < IL::kSize) L.in[buf ^ 1][e] = pre[u];
      }
    }
    ASVRL_STAMP(12);
    __syncthreads();
    ASVRL_STAMP(13);

    // ---------------- dW1[own][:] += dz1^T x; L4's first weight fragments fetched meanwhile
    frag8 wt[8], wcc[4];
    {
      ASVRL_FRESH_LANE();
      const TrA<kH> TA_d = tr_base<kH, LT>(LB, lane);
      const TrA<kC> TA_x = tr_base<kC, LT>(LB, lane);
#pragma unroll
      for (int ks = 0; ks < 8; ++ks) wt[ks] = W1T[((2 * w) * 8 + ks) * 64 + lane];
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) wcc[ks] = WCR ? wcr0[ks] : WC[((2 * w) * 4 + ks) * 64 + lane];
        mfma_grid<G / 16, 8>([&](int kk) { return trf(L.dz1, TA_d, kk, w); },
                             [&](int kk, int n) { return trf(L.x, TA_x, kk, n); },
                             [&](int kk, int n, const frag8& A, const frag8& B) {
                               if (n == 0) db1 += sum8(A);
                               mfma_acc(dW1[n], A, B);
                             });
      ASVRL_STAMP(22);
    }
    if constexpr (AH) {   // round t + grid's images, behind the dW1 MFMAs
      const int tn = t + static_cast<int>(gridDim.x);
      if (tn < a.rounds) stage(tn * G / NT, L.in[buf ^ 1], L.cos[buf ^ 1], L.F[buf ^ 1], L.G[buf ^ 1]);
    }
    ASVRL_STAMP(23);

    // ---------------- L4: dx = W1^T dz1 (own blocks 2w, 2w+1) with c = relu(Wc cos + bc) recomputed
    // (bit-identical to L0's); dF = sum over taus of dx c (-> dzF), dzc = dx F 1[c > 0] into the
    // wave's own dzc image. No barrier: L4 reads dz1 and cos, which nothing writes this round any more.
#pragma unroll
    for (int mq = 0; mq < 2; ++mq) {
      ASVRL_FRESH_LANE();
      const RowA<kNcos> RA_cos = row_base<kNcos, LT>(LB, lane, r, h);
      const RowA<kH> RA_d = row_base<kH, LT>(LB, lane, r, h);
      const RowA<kNcos> RA_dzc = row_base<kNcos, LT>(LB, lane, r, h);
      const int mb = 2 * w + mq;
      float fv[NB][2][8];
#pragma unroll
      for (int j = 0; j < NB; ++j)
#pragma unroll
        for (int s = 0; s < 2; ++s) lds8(Fb + ((32 * j + r) / NT) * kC + mb * 32 + 16 * s + 8 * h, fv[j][s]);
      float fsa[NB][16];
      f32x16 dxs[ASVRL_READ_AHEAD ? NB : 1], ccs[ASVRL_READ_AHEAD ? NB : 1];
      if constexpr (ASVRL_READ_AHEAD != 0) {
#pragma unroll
        for (int j = 0; j < NB; ++j) {
          dxs[j] = f32x16{};
          ccs[j] = acc_init(bcp, mb * 32, h);
        }
        mfma_rows<8, NB>(dxs, L.dz1, RA_d, [&](int ks) { return wt[ks]; });
        mfma_rows<4, NB>(ccs, cosb, RA_cos, [&](int ks) { return wcc[ks]; });
      }
      ASVRL_STAMP(24 + 3 * mq);
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        f32x16 dx, cc;
        if constexpr (ASVRL_READ_AHEAD != 0) {
          dx = dxs[ASVRL_READ_AHEAD ? j : 0];
          cc = ccs[ASVRL_READ_AHEAD ? j : 0];
        } else {
          dx = f32x16{};
#pragma unroll
          for (int ks = 0; ks < 8; ++ks) dx = mfma(wt[ks], rowf(L.dz1, RA_d, j, ks), dx);
          cc = acc_init(bcp, mb * 32, h);
#pragma unroll
          for (int ks = 0; ks < 4; ++ks) cc = mfma(wcc[ks], rowf(cosb, RA_cos, j, ks), cc);
        }
        if constexpr (!kBiasFirst) cc += bias_init(bcp, mb * 32, h);
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          float cv[8], d[8], fs[8], df[8], dz[8];
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            cv[i] = relu(cc[8 * s + i]);
            d[i] = dx[8 * s + i];
          }
          mul8(d, cv, fs);
          mul8(d, fv[j][s], df);
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            fsa[j][8 * s + i] = fs[i];
            dz[i] = cv[i] > 0.f ? df[i] : 0.f;
          }
          rows(dzc_w, RA_dzc, j, 2 * mq + s, pack8(dz));
        }
      }
      if (mq == 0) {   // the second block's fragments
#pragma unroll
        for (int ks = 0; ks < 8; ++ks) wt[ks] = W1T[((2 * w + 1) * 8 + ks) * 64 + lane];
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) wcc[ks] = WCR ? wcr1[ks] : WC[((2 * w + 1) * 4 + ks) * 64 + lane];
      }
      ASVRL_STAMP(25 + 3 * mq);
      sample_sums<NT, NB>(fsa, mb * 32, lane, [&](int bl, int p, float v) {
        const float fm = Fb[bl * kC + p];
        const float dz = fm > 0.f ? v : 0.f;
        if (a.dzF != nullptr) bp(a.dzF)[static_cast<size_t>(b0 + bl) * kC + swap23(p)] = (elem_t)dz;
        if (a.parts.enc != nullptr) Fb[bl * kC + p] = dz;   // F's blocks 2w, 2w+1 are this wave's own
      });
      ASVRL_STAMP(26 + 3 * mq);
    }
    {
      if (a.parts.enc != nullptr) {
        // the observation encoders' gradients (AC_IQN_model.py:284-308): lane l owns feature
        // m = swap23(64 w + l) and sums dzF[b][m] * (its encoder's inputs, 1) over the round's samples
        // in order; object features keep their object's slot (folded over the objects at the end)
        ASVRL_FRESH_LANE();
        const int p = 64 * w + lane, m = swap23(p);
        const bool self = m < kSelfF;
        const int off = self ? 0 : kSelfIn + kObjIn * ((m - kSelfF) / kObjF);
        float acc[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i] = 0.f;
#pragma unroll
        for (int k = 0; k < S; ++k) {
          const float d = Fb[k * kC + p];
          const float* x = in + IL::kObs + k * kObsIn + off;
#pragma unroll
          for (int i = 0; i < kSelfIn; ++i) acc[i] += d * ((self || i < kObjIn) ? x[i] : 0.f);
          acc[7] += d;
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          if constexpr (IQN) encr[i] += acc[i];   // IQN: no LDS to spare at N = 8, VGPRs to spare
          else L.encacc[i * kC + m] += acc[i];
        }
      }
    }

    ASVRL_STAMP(30);
    // ---------------- dWc[own 64][:] += dzc^T cos (this wave's own dzc image: in-order LDS, no barrier)
    {
      ASVRL_FRESH_LANE();
      const TrA<kNcos> TA_cos = tr_base<kNcos, LT>(LB, lane);
      const TrA<kNcos> TA_dzc = tr_base<kNcos, LT>(LB, lane);
#pragma unroll
        for (int kk = 0; kk < G / 16; ++kk) {
          const frag8 A0 = trf(dzc_w, TA_dzc, kk, 0);
          const frag8 A1 = trf(dzc_w, TA_dzc, kk, 1);
          dbc0 += sum8(A0);
          dbc1 += sum8(A1);
#pragma unroll
          for (int n = 0; n < 2; ++n) {
            const frag8 Bf = trf(cosb, TA_cos, kk, n);
            mfma_acc(dWc[n], A0, Bf);
            mfma_acc(dWc[2 + n], A1, Bf);
          }
        }
    }
    if constexpr (!AH) {
#pragma unroll
      for (int u = 0; u < IL::kPer; ++u) {
        const int e = tid_p + u * kNW * 64;
        if (e < IL::kSize) L.in[buf ^ 1][e] = pre[u];
      }
    }
    ASVRL_STAMP(14);
    __syncthreads();   // the next round overwrites cos, F, G, x, a, b, dz1
    ASVRL_STAMP(15);
  }

  // ---------------- the workgroup's partials: [M*K + M] per layer, features in natural order
  mfma_drain();
  {
    // encoders (the round loop ended on a barrier: every wave's sums are in LDS; IQN's are moved from
    // registers into the x image, free now). Object features folded over the five objects in object
    // order; the action encoder's two lane halves in order.
    const float* ea = L.encacc;
    if constexpr (IQN) {
      if (a.parts.enc != nullptr) {
        float* ex = reinterpret_cast<float*>(L.x);
        const int m = swap23(64 * w + lane);
#pragma unroll
        for (int i = 0; i < 8; ++i) ex[i * kC + m] = encr[i];
        ea = ex;
      }
      __syncthreads();
    }
    if (a.parts.enc != nullptr) {
      float* pe = a.parts.enc + static_cast<size_t>(grp) * 688;
      for (int i = threadIdx.x; i < 688; i += kNW * 64) {
        float v;
        if (i < kSelfF * kSelfIn) v = ea[(i % kSelfIn) * kC + i / kSelfIn];
        else if (i < kSelfF * (kSelfIn + 1)) v = ea[7 * kC + i - kSelfF * kSelfIn];
        else {
          const int e = i - kSelfF * (kSelfIn + 1);
          const int j = e < kObjF * kObjIn ? e / kObjIn : e - kObjF * kObjIn;
          const int slot = e < kObjF * kObjIn ? e % kObjIn : 7;
          v = 0.f;
#pragma unroll
          for (int o = 0; o < 5; ++o) v += ea[slot * kC + kSelfF + kObjF * o + j];
        }
        pe[i] = v;
      }
    }
    if (!IQN && a.parts.aenc != nullptr) {
      float* pa = a.parts.aenc + static_cast<size_t>(grp) * (3 * kH);
      for (int i = threadIdx.x; i < 3 * kH; i += kNW * 64) {
        const int m = i < 2 * kH ? i / 2 : i - 2 * kH, c = i < 2 * kH ? i % 2 : 2;
        pa[i] = L.aeacc[(2 * c) * kH + m] + L.aeacc[(2 * c + 1) * kH + m];
      }
    }
  }
  float* p2 = a.parts.hidden2 + static_cast<size_t>(grp) * (kH * kH + kH);
  float* p1 = a.parts.hidden + static_cast<size_t>(grp) * (kH * kC + kH);
  float* pc = a.parts.cos_emb + static_cast<size_t>(grp) * (kC * kNcos + kC);
#pragma unroll
  for (int g = 0; g < 16; ++g) {
    const int m = (g & 3) + 8 * (g >> 2) + 4 * h;   // MFMA C row of register g
    const int f2 = swap23(w * 32 + m);
#pragma unroll
    for (int n = 0; n < 4; ++n) p2[f2 * kH + swap23(32 * n + r)] = dW2[n][g];
#pragma unroll
    for (int n = 0; n < 8; ++n) p1[f2 * kC + swap23(32 * n + r)] = dW1[n][g];
#pragma unroll
    for (int mq = 0; mq < 2; ++mq) {
      const int fc = swap23((2 * w + mq) * 32 + m);
#pragma unroll
      for (int n = 0; n < 2; ++n) pc[fc * kNcos + 32 * n + r] = dWc[mq * 2 + n][g];
    }
  }
  dbc0 = half_sum(dbc0);
  dbc1 = half_sum(dbc1);
  db2 = half_sum(db2);
  db1 = half_sum(db1);
  if (h == 0) {
    p2[kH * kH + swap23(w * 32 + r)] = db2;
    p1[kH * kC + swap23(w * 32 + r)] = db1;
    pc[kC * kNcos + swap23(2 * w * 32 + r)] = dbc0;
    pc[kC * kNcos + swap23((2 * w + 1) * 32 + r)] = dbc1;
  }
  if constexpr (IQN) {
    // output layer [32 actions][128] + [32]: register g = action row, lane = feature position
    float* po = a.parts.out + static_cast<size_t>(grp) * (kMaxA * kH + kMaxA);
#pragma unroll
    for (int g = 0; g < 16; ++g) po[((g & 3) + 8 * (g >> 2) + 4 * h) * kH + swap23(w * 32 + r)] = dWo[g];
    dbo = half_sum(dbo);   // lane r: the action r column's sum over the round rows (every wave alike)
    if (w == 0 && h == 0) po[kMaxA * kH + r] = dbo;
    return;
  }
  // output layer: sum over the half's 32 lanes (rows) of each register (feature), then the waves' dbo
  float* po = a.parts.out + static_cast<size_t>(grp) * (kH + 1);
#pragma unroll
  for (int g = 0; g < 16; ++g) {
    const float v = seg_sum<32>(dwo[IQN ? 0 : g]);   // lane 31 of each half
    if (r == 31) po[swap23(w * 32 + 16 * (g >> 3) + 8 * h + (g & 7))] = v;
  }
  dbo = seg_sum<32>(h == 0 ? dbo : 0.f);
  if (lane == 31) L.red[w] = dbo;
  __syncthreads();
  if (threadIdx.x == 0) po[kH] = ((L.red[0] + L.red[1]) + L.red[2]) + L.red[3];
}

#if !ASVRL_OPERAND_F32
// =================================================================================================================
// critic_fused8_kernel -- the same critic update (and, TQ, the target critic's forward) at TWO waves per SIMD:
// 8 waves, 512 threads per workgroup, one workgroup per CU. VERDICT r05 item 1: at one wave per SIMD the round was
// vector-issue and latency bound (MFMA busy ~20 %: a lone wave issues one VALU instruction per 4 cycles and nothing
// covers its LDS / L2 waits); two waves per SIMD issue VALU at the SIMD's full rate (2 cycles per wave instruction)
// and one wave's MFMAs run while its partner issues its epilogue. The register file is split in half: each wave owns
// HALF of the persistent weight-gradient accumulators (128 AGPRs instead of 256) and has 128 VGPRs for the round.
//
// Wave v: w = v & 3 (the feature block the old kernel's wave w owned), j = v >> 2 (the half). Waves w and w + 4 share
// a SIMD (the workgroup's waves go round the four SIMDs) and split the old wave w's work:
//   L0, L4, dzc, dWc (256 cos-layer features)  by feature:  cos block cb = 2w + j, both row blocks;
//   L1 (K = 256)                               by K:        hidden block w, k-steps 8j..8j+7, both row blocks;
//                                                           the partner's partial sum of row block j is added
//                                                           through LDS (the free dzc images) before the epilogue;
//   L2, dz2, L3 (128 features)                 by rows:     hidden block w, row block j (= sample j at N = 32);
//   dW2 / dW1 (rows = own features)            by columns:  n in {2j, 2j+1} / {4j .. 4j+3};
//   loss                                        waves 0-3 (16-row groups, as before).
// AGPRs per wave: dW2 2 + dW1 4 + dWc 2 blocks of 16 = 128. Per-sample sums over a row block (dG, dF) reduce 16
// values over the 32 lanes of a half (half_rows_sum16); the output layer's gradient is reduced per round.
// One barrier more per round than critic_fused_kernel (the L1 partial exchange).
//
// The target pass (TQ) runs the SAME forward phases (L0, L1, L2) on the target critic's weights, round by round over
// the workgroup's own samples, and stores q_next for the update's rounds (global, read back by this workgroup after
// the barrier); the target's biases and encoders occupy the LDS slots of the local ones until the update starts.
//
// Shapes: AC-IQN, N = N' = 32, bf16 operands, the encoders' gradients in the launch (parts.enc / parts.aenc), no
// per-sample dzF / dzG / xb outputs; critic_fused_kernel takes every other case. Same rounding points as
// critic_fused_kernel (checked against oracle/learn_ref.critic_step_bf16 / critic_forward_bf16); the f32
// summation order differs (L1's two K halves, the per-round row sums), so the two kernels agree within f32
// rounding, not bit for bit.
constexpr int kNW8 = 8, kT8 = kNW8 * 64;

// sum of each of 16 values over the 32 lanes of each lane half: afterwards x[0] of lane r (either 16-lane row of
// the half) holds the sum of value r % 16 (transpose-reduce over lane bits 0..3, then the two rows)
__device__ __forceinline__ void half_rows_sum16(float (&x)[16], int lane) {
  xreduce<16, 16>(x, lane);
  x[0] = row_pair_sum(x[0]);
}

// the same for 8 values: x[0] of lane r holds the sum of value r % 8 (lane bits 0..2, then bit 3 by a row rotation
// of 8 -- lane ^ 8 inside its 16-lane row -- then bit 4)
__device__ __forceinline__ void half_rows_sum8(float (&x)[8], int lane) {
  xreduce<8, 8>(x, lane);
  x[0] += dpp<0x128>(x[0]);   // row_ror:8
  x[0] = row_pair_sum(x[0]);
}

// F (observation_processor) and G (relu(action_encoder(a))) of the round's 2 samples: thread t computes feature
// t & 255 of sample t >> 8 (stage_fg's arithmetic, op for op, uncontracted)
__device__ __forceinline__ void stage_fg8(int tid, const float* in, int kact, const float* enc, float* Fs, float* Gs) {
#pragma clang fp contract(off)
  const float* self_w = enc;
  const float* self_b = self_w + 56 * 7;
  const float* obj_w = self_b + 56;
  const float* obj_b = obj_w + 40 * 5;
  const float* ae_w = obj_b + 40;
  const float* ae_b = ae_w + 128 * 2;
  const int m = tid & 255, k = tid >> 8;
  const float* x = in + k * kObsIn;
  float v;
  if (m < kSelfF) {
    float d = 0.f;
#pragma unroll
    for (int i = 0; i < kSelfIn; ++i) d += self_w[m * kSelfIn + i] * x[i];
    v = relu(d + self_b[m]);
  } else {
    const int o = (m - kSelfF) / kObjF, jf = (m - kSelfF) % kObjF;
    const float* xo = x + kSelfIn + kObjIn * o;
    float d = 0.f;
#pragma unroll
    for (int i = 0; i < kObjIn; ++i) d += obj_w[jf * kObjIn + i] * xo[i];
    v = x[kObsMask + o] < 0.5f ? 0.f : relu(d + obj_b[jf]);   // masked_fill(mask < 0.5, 0)
  }
  Fs[k * kC + swap23(m)] = static_cast<float>((elem_t)v);
  if (m < kH)
    Gs[k * kH + swap23(m)] = relu((ae_w[2 * m] * in[kact + 2 * k] + ae_w[2 * m + 1] * in[kact + 2 * k + 1]) + ae_b[m]);
}

// element e (< kObs + kAct + kTau) of the TARGET pass's round t inputs: next observation rows, next actions, taus'
template <class IL>
__device__ __forceinline__ float fetch_tq(const ctile::CriticArgs& t, int r, int e) {
  constexpr int S = 2, G = 64;
  const int64_t b0 = static_cast<int64_t>(r) * S;
  const float* p;
  if (e < IL::kAct) p = t.obs + (b0 + e / kObsIn) * t.ld_obs + e % kObsIn;
  else if (e < IL::kTau) p = t.ain + (b0 + (e - IL::kAct) / 2) * t.ld_ain + (e - IL::kAct) % 2;
  else p = t.taus + static_cast<int64_t>(r) * G + (e - IL::kTau);
  return *p;
}

template <bool TQ>
__global__ __launch_bounds__(kT8) __attribute__((amdgpu_waves_per_eu(2, 2)))
void critic_fused8_kernel(FusedArgs a) {
  constexpr int NT = 32, NB = 2, G = 64, S = 2;
  using IL = InLayout<NT, S, G, 2>;
  constexpr int kPer8 = (IL::kSize + kT8 - 1) / kT8;
  __shared__ __attribute__((aligned(16))) FusedLds<NT, NB, S, false, 2> L;
  __shared__ int LB[kLbFields][64];
  __shared__ __attribute__((aligned(16))) float red8[2][kH];   // the output layer's gradient, one row per half
  static_assert(sizeof(L) + sizeof(LB) + sizeof(red8) <= 160 * 1024, "fused8 LDS exceeds the CU's 160 KB");
  // the L1 partial exchange: [w][row block][4 quarters][64 lanes] f32x4 in the dzc images (free until L4)
  static_assert(sizeof(L.dzc) >= 4 * 2 * 16 * 64 * 4, "L1 exchange scratch");
  float* const xch = reinterpret_cast<float*>(&L.dzc[0][0]);
  {
    const int lane = threadIdx.x & 63, h = lane >> 5, r = lane & 31;
    if (threadIdx.x < 64) {
      LB[kLbR64][lane] = RowA<kNcos>(r, h).base;
      LB[kLbR128][lane] = RowA<kH>(r, h).base;
      LB[kLbR256][lane] = RowA<kC>(r, h).base;
      const auto t64 = TrA<kNcos>(lane);
      const auto t128 = TrA<kH>(lane);
      const auto t256 = TrA<kC>(lane);
      LB[kLbT64lo][lane] = t64.lo;
      LB[kLbT64hi][lane] = t64.hi;
      LB[kLbT128lo][lane] = t128.lo;
      LB[kLbT128hi][lane] = t128.hi;
      LB[kLbT256lo][lane] = t256.lo;
      LB[kLbT256hi][lane] = t256.hi;
    }
  }
  float* const bcp = L.bias;
  float* const b1p = L.bias + kC;
  float* const b2p = L.bias + kC + kH;
  float* const wop = L.bias + kC + 2 * kH;
  // biases (position order), wo, bo and the encoders of weight set `ws` into LDS
  auto load_params = [&](const AsvCriticWeights& ws) {
    for (int i = threadIdx.x; i < kC; i += kT8) bcp[swap23(i)] = ws.bc[i];
    for (int i = threadIdx.x; i < kH; i += kT8) {
      b1p[swap23(i)] = ws.b1[i];
      b2p[swap23(i)] = ws.b2[i];
      wop[swap23(i)] = ws.wo[i];
    }
    if (threadIdx.x == 0) L.bias[kC + 3 * kH] = ws.bo[0];
    constexpr int kEncPer = (kEncFloats + kT8 - 1) / kT8;
    float ev[kEncPer];
#pragma unroll
    for (int u = 0; u < kEncPer; ++u) {
      int e = threadIdx.x + u * kT8;
      const float* src = ws.self_w;
      if (e >= 392) { e -= 392; src = ws.self_b;
        if (e >= 56) { e -= 56; src = ws.obj_w;
          if (e >= 200) { e -= 200; src = ws.obj_b;
            if (e >= 40) { e -= 40; src = ws.ae_w;
              if (e >= 256) { e -= 256; src = ws.ae_b; } } } } }
      ev[u] = threadIdx.x + u * kT8 < kEncFloats ? src[e] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < kEncPer; ++u)
      if (threadIdx.x + u * kT8 < kEncFloats) L.enc[threadIdx.x + u * kT8] = ev[u];
  };
  // F, G and cos(tau pi k) of a round (inputs staged at `ins`) into one image set; targets r + gamma q' (1 - d) in
  // place over q' unless `fwd_only`
  auto stage = [&](float* ins, elem_t* cosd, float* Fd, float* Gd, bool fwd_only) {
    int tid_s = threadIdx.x;
    asm volatile("" : "+v"(tid_s));
    stage_fg8(tid_s, ins, IL::kAct, L.enc, Fd, Gd);
    if (!fwd_only && tid_s < S * NT) {
      const int k = tid_s / NT;
      float* qn = ins + IL::kQn + tid_s;
      *qn = ins[IL::kRew + k] + (a.gamma * *qn) * (1.0f - ins[IL::kDon + k]);
    }
    static_assert(G * (kNcos / 8) == kT8, "one cos chunk per thread");
    const int row = tid_s / (kNcos / 8), ch = tid_s % (kNcos / 8);
    float cv[8];
    cos_pi_k_tau8r(ins[IL::kTau + row], 8 * ch, cv);
    row_store<kNcos>(cosd, row, 8 * ch, pack8(cv));
  };

  // ---------------- the forward phases, on weight set `ws` (local or target)
  // L0: c = relu(Wc cos + bc), x = F c for cos block cb = 2w + j, both row blocks
  // the Wc fragments of cos block cb (4) and, fetched here for L1a, the wave's W1 half (8)
  auto load_wc = [&](const AsvCriticWeights& ws, frag8 (&wc)[4]) {
    ASVRL_FRESH_LANE();
    const int v = __builtin_amdgcn_readfirstlane(tid_ >> 6);
    const int cb = 2 * (v & 3) + (v >> 2);
    const frag8* WC = reinterpret_cast<const frag8*>(ws.wc_frag);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) wc[ks] = WC[(cb * 4 + ks) * 64 + lane];
  };
  auto phase_L0 = [&](const AsvCriticWeights& ws, const frag8 (&wc)[4], const elem_t* cosb, const float* Fb,
                      frag8 (&w1f)[8]) {
    ASVRL_FRESH_LANE();
    const int v = __builtin_amdgcn_readfirstlane(tid_ >> 6);
    const int w = v & 3, j = v >> 2, cb = 2 * w + j;
    const RowA<kNcos> RA_cos = row_base<kNcos, true>(LB, lane, r, h);
    const RowA<kC> RA_x = row_base<kC, true>(LB, lane, r, h);
    frag8 cf[4];   // one row block's cos operands at a time (the next block's read behind this one's MFMAs)
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) cf[ks] = rowf(cosb, RA_cos, 0, ks);
#pragma unroll
    for (int rb = 0; rb < NB; ++rb) {
      f32x16 acc = acc_init(bcp, cb * 32, h);
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) acc = mfma(wc[ks], cf[ks], acc);
      __builtin_amdgcn_sched_barrier(0);
      if (rb + 1 < NB) {
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) cf[ks] = rowf(cosb, RA_cos, rb + 1, ks);
      } else {   // L1a's fragments, behind the last block's MFMAs
        const frag8* W1 = reinterpret_cast<const frag8*>(ws.w1_frag);
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) w1f[kk] = W1[(w * 16 + 8 * j + kk) * 64 + lane];
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        float fv[8], cv[8], xv[8];
        lds8(Fb + rb * kC + cb * 32 + 16 * s + 8 * h, fv);
#pragma unroll
        for (int i = 0; i < 8; ++i) cv[i] = acc[8 * s + i];
        mul8(fv, cv, xv);
        rows(L.x, RA_x, rb, 2 * cb + s, relu_packed(pack8(xv)));   // F >= 0: relu of the packed product
      }
    }
  };
  // L1, first half: block w over k-steps 8j..8j+7 for both row blocks; the partial of row block 1 - j to the
  // exchange slot, row block j's kept in `keep`
  auto phase_L1a = [&](const AsvCriticWeights& ws, const frag8 (&w1f)[8], f32x16& keep, frag8 (&w2f)[8]) {
    ASVRL_FRESH_LANE();
    const int v = __builtin_amdgcn_readfirstlane(tid_ >> 6);
    const int w = v & 3, j = v >> 2;
    const RowA<kC> RA_x = row_base<kC, true>(LB, lane, r, h);
    f32x16 acc[NB];
    const f32x16 b0 = acc_init(b1p, w * 32, h);
#pragma unroll
    for (int rb = 0; rb < NB; ++rb) acc[rb] = j == 0 ? b0 : f32x16{};
    // k-steps 8j + kk: the chained image's 16-byte chunk 2 (8j + kk) + h lies 256 j bytes further in the row
    mfma_rows<8, NB>(acc, L.x + 128 * j, RA_x, [&](int kk) { return w1f[kk]; });
    {   // L2's fragments, behind the MFMAs
      const frag8* W2 = reinterpret_cast<const frag8*>(ws.w2_frag);
#pragma unroll
      for (int ks = 0; ks < 8; ++ks) w2f[ks] = W2[(w * 8 + ks) * 64 + lane];
    }
    const f32x16 give = j ? acc[0] : acc[1];
    keep = j ? acc[1] : acc[0];
    float* dst = xch + ((w * 2 + (1 - j)) * 4) * 256 + lane * 4;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      *reinterpret_cast<f32x4*>(dst + q * 256) = f32x4{give[4 * q], give[4 * q + 1], give[4 * q + 2], give[4 * q + 3]};
  };
  // L1, second half: + the partner's partial; h1 = relu(.), h1g = h1 G (row block j = sample j); returns h1
  // (packed) for L3's mask
  auto phase_L1b = [&](f32x16 keep, const float* Gb, frag8 (&h1k)[2]) {
    ASVRL_FRESH_LANE();
    const int v = __builtin_amdgcn_readfirstlane(tid_ >> 6);
    const int w = v & 3, j = v >> 2;
    const float* src = xch + ((w * 2 + j) * 4) * 256 + lane * 4;
    float gv[2][8];
#pragma unroll
    for (int s = 0; s < 2; ++s) lds8(Gb + j * kH + w * 32 + 16 * s + 8 * h, gv[s]);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const f32x4 o = *reinterpret_cast<const f32x4*>(src + q * 256);
#pragma unroll
      for (int i = 0; i < 4; ++i) keep[4 * q + i] += o[i];
    }
    const RowA<kH> RA_a = row_base<kH, true>(LB, lane, r, h);
    elem_t* const arow = L.a + j * 32 * kH;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      float hv[8], gov[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) hv[i] = relu(keep[8 * s + i]);
      h1k[s] = pack8(hv);
      mul8(hv, gv[s], gov);
      rows(arow, RA_a, 0, 2 * w + s, pack8(gov));
    }
  };
  // L2: z2 = W2 h1g + b2 for block w, row block j; partial q over the block's features into qpart; h2 parked in b
  auto phase_L2 = [&](const frag8 (&w2f)[8], const frag8* W2T, frag8 (&w2tf)[8]) {
    ASVRL_FRESH_LANE();
    const int v = __builtin_amdgcn_readfirstlane(tid_ >> 6);
    const int w = v & 3, j = v >> 2;
    const RowA<kH> RA_a = row_base<kH, true>(LB, lane, r, h);
    f32x16 z2[1] = {acc_init(b2p, w * 32, h)};
    mfma_rows<kH / 16, 1>(z2, L.a + j * 32 * kH, RA_a, [&](int ks) { return w2f[ks]; });
    if (W2T != nullptr)   // L3's fragments (the update only)
#pragma unroll
      for (int ks = 0; ks < 8; ++ks) w2tf[ks] = W2T[(w * 8 + ks) * 64 + lane];
    float wov[2][8];
#pragma unroll
    for (int s = 0; s < 2; ++s) lds8(wop + w * 32 + 16 * s + 8 * h, wov[s]);
    float part = 0.f;
    elem_t* const brow = L.b + j * 32 * kH;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      float hv[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float h2 = relu(z2[0][8 * s + i]);
        part += wov[s][i] * h2;
        hv[i] = h2;
      }
      rows(brow, RA_a, 0, 2 * w + s, pack8(hv));
    }
    part = half_sum(part);
    if (h == 0) L.qpart[w][32 * j + r] = part;
  };

  // ---------------- the target critic's forward (TQ): q_next of the workgroup's own samples
  if constexpr (TQ) {
    load_params(a.tq.w);
    __syncthreads();
    frag8 wct[4];
    load_wc(a.tq.w, wct);
    for (int t = blockIdx.x; t < a.rounds; t += gridDim.x) {
      for (int e = threadIdx.x; e < IL::kQn; e += kT8) L.in[0][e] = fetch_tq<IL>(a.tq, t, e);
      __syncthreads();
      stage(L.in[0], L.cos[0], L.F[0], L.G[0], true);
      __syncthreads();
      frag8 w1f[8], w2f[8], unused[8];
      phase_L0(a.tq.w, wct, L.cos[0], L.F[0], w1f);
      f32x16 keep;
      __syncthreads();
      phase_L1a(a.tq.w, w1f, keep, w2f);
      __syncthreads();
      frag8 h1k[2];
      phase_L1b(keep, L.G[0], h1k);
      __syncthreads();
      phase_L2(w2f, nullptr, unused);
      __syncthreads();
      if (threadIdx.x < G) {
        const int lr = threadIdx.x;
        a.tq.q[static_cast<int64_t>(t) * G + lr] =
            (((L.qpart[0][lr] + L.qpart[1][lr]) + L.qpart[2][lr]) + L.qpart[3][lr]) + L.bias[kC + 3 * kH];
      }
    }
    __syncthreads();   // every q_next of the workgroup stored; the LDS is the update's from here
  }

  // ---------------- the update: local parameters, the first round's inputs, its images
  load_params(a.w);
  for (int i = threadIdx.x; i < 8 * kC; i += kT8) L.encacc[i] = 0.f;
  for (int i = threadIdx.x; i < 3 * 2 * kH; i += kT8) L.aeacc[i] = 0.f;
  if (blockIdx.x < a.rounds)
#pragma unroll
    for (int u = 0; u < kPer8; ++u) {
      const int e = threadIdx.x + u * kT8;
      if (e < IL::kSize) L.in[0][e] = fetch_in<NT, S, G, 2>(a, blockIdx.x, e);
    }
  __syncthreads();
  if (blockIdx.x < a.rounds) stage(L.in[0], L.cos[0], L.F[0], L.G[0], false);
  __syncthreads();

  f32x16 dW2[2], dW1[4], dWc[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) dW2[i] = dWc[i] = f32x16{};
#pragma unroll
  for (int i = 0; i < 4; ++i) dW1[i] = f32x16{};
  float db2 = 0.f, db1 = 0.f, dbc = 0.f, dbo = 0.f, dwo1 = 0.f;
  frag8 wcr[4];   // cos block cb's Wc fragments (L0; reloaded in each round's dW1 phase for L4 and the next L0)
  load_wc(a.w, wcr);
  int buf = 0;
  for (int t = blockIdx.x; t < a.rounds; t += gridDim.x, buf ^= 1) {
    float pre[kPer8];
    int tid_p = threadIdx.x;
    asm volatile("" : "+v"(tid_p));
    float* const in = L.in[buf];
    const int row0 = t * G, b0 = row0 / NT;
    (void)b0;
    elem_t* const cosb = L.cos[buf];
    float* const Fb = L.F[buf];
    float* const Gb = L.G[buf];

    frag8 w1f[8], w2f[8], w2tf[8];
    phase_L0(a.w, wcr, cosb, Fb, w1f);
    __syncthreads();
    f32x16 keep;
    phase_L1a(a.w, w1f, keep, w2f);
    // the next round's inputs into registers (stored to LDS before the dW1 phase stages them)
#pragma unroll
    for (int u = 0; u < kPer8; ++u) {
      const int e = tid_p + u * kT8;
      pre[u] = (t + static_cast<int>(gridDim.x) < a.rounds && e < IL::kSize)
                   ? fetch_in<NT, S, G, 2>(a, t + gridDim.x, e) : 0.f;
    }
    __syncthreads();
    frag8 h1k[2];
    phase_L1b(keep, Gb, h1k);
    __syncthreads();
    phase_L2(w2f, nullptr, w2tf);
    __syncthreads();

    // ---------------- loss (waves 0-3): q = sum of the four partials + bo; quantile-Huber -> dq
    {
      ASVRL_FRESH_LANE();
      const int v = __builtin_amdgcn_readfirstlane(tid_ >> 6);
      if (v < 4) {
        const int q4 = lane >> 4;
        const int g = v;
        const int lr = 16 * g + (lane & 15), grow = row0 + lr, bl = lr / NT;
        const float bo = L.bias[kC + 3 * kH];
        const float q = (((L.qpart[0][lr] + L.qpart[1][lr]) + L.qpart[2][lr]) + L.qpart[3][lr]) + bo;
        float wl;
        const float dq = quarter_loss_dq<NT>(a, in + IL::kQn + bl * NT, in[IL::kTau + lr], q, q4, &wl);
        if (a.tile_loss != nullptr) {
          const float sv = seg_sum<16>(wl);
          if (lane == 0) L.tsum[g] = sv;
        }
        if (q4 == 0) {
          L.dq[lr] = dq;
          if (a.row_loss != nullptr) a.row_loss[grow] = wl;
          if (a.q != nullptr) a.q[grow] = q;
          dbo += dq;
        }
      }
    }
    __syncthreads();

    // ---------------- dz2 = dq wo 1[h2 > 0] (block w, row block j, in place over h2); the output layer's gradient
    // sum dq h2 over the row block
    if (a.tile_loss != nullptr && threadIdx.x < G / 32)
      a.tile_loss[row0 / 32 + threadIdx.x] = (L.tsum[2 * threadIdx.x] + L.tsum[2 * threadIdx.x + 1]) * a.loss_scale;
    {
      ASVRL_FRESH_LANE();
      const int v = __builtin_amdgcn_readfirstlane(tid_ >> 6);
      const int w = v & 3, j = v >> 2;
      {   // L3's fragments, one phase ahead
        const frag8* W2T = reinterpret_cast<const frag8*>(a.w.w2t_frag);
#pragma unroll
        for (int ks = 0; ks < 8; ++ks) w2tf[ks] = W2T[(w * 8 + ks) * 64 + lane];
      }
      const RowA<kH> RA_b = row_base<kH, true>(LB, lane, r, h);
      elem_t* const brow = L.b + j * 32 * kH;
      float wov[2][8];
#pragma unroll
      for (int s = 0; s < 2; ++s) lds8(wop + w * 32 + 16 * s + 8 * h, wov[s]);
      const float dqv = L.dq[32 * j + r];
      frag8 hv[2];
#pragma unroll
      for (int s = 0; s < 2; ++s) hv[s] = rowf(brow, RA_b, 0, 2 * w + s);
      float pr[16];
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        float dz[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          dz[i] = dqv * wov[s][i];
          pr[8 * s + i] = dqv * static_cast<float>(hv[s][i]);
        }
        rows(brow, RA_b, 0, 2 * w + s, mask_pos(pack8(dz), hv[s]));   // dq wo 1[h2 > 0]
      }
      half_rows_sum16(pr, lane);
      dwo1 += pr[0];
    }
    __syncthreads();

    // ---------------- L3: dh1g = W2^T dz2 (block w, row block j) -> dz1, dG;  dW2[own][2j, 2j+1] += dz2^T h1g
    {
      ASVRL_FRESH_LANE();
      const int v = __builtin_amdgcn_readfirstlane(tid_ >> 6);
      const int w = v & 3, j = v >> 2;
      const RowA<kH> RA = row_base<kH, true>(LB, lane, r, h);
      float gv[2][8];
#pragma unroll
      for (int s = 0; s < 2; ++s) lds8(Gb + j * kH + w * 32 + 16 * s + 8 * h, gv[s]);
      f32x16 acc[1] = {f32x16{}};
      mfma_rows<kH / 16, 1>(acc, L.b + j * 32 * kH, RA, [&](int ks) { return w2tf[ks]; });
      pin(h1k[0]);
      pin(h1k[1]);
      float gsa[16];
      elem_t* const drow = L.dz1 + j * 32 * kH;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        float h1[8], d[8], dg[8], hd[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          h1[i] = static_cast<float>(h1k[s][i]);
          d[i] = acc[0][8 * s + i];
        }
        mul8(d, gv[s], dg);
        mul8(d, h1, hd);
#pragma unroll
        for (int i = 0; i < 8; ++i) gsa[8 * s + i] = hd[i];
        rows(drow, RA, 0, 2 * w + s, mask_pos(pack8(dg), h1k[s]));   // dz1 = dh1g G 1[h1 > 0]
      }
      // dG of sample j = sum over its 32 taus of dh1g h1 -> dzG = dG 1[G > 0], in place over G's block w
      half_rows_sum16(gsa, lane);
      if (r < 16) {
        const int p = w * 32 + 16 * (r >> 3) + 8 * h + (r & 7);
        const float gm = Gb[j * kH + p];
        Gb[j * kH + p] = gm > 0.f ? gsa[0] : 0.f;
      }
      // action_encoder's gradient (AC_IQN_model.py:468-470): lanes of half 0 (feature 32 w + r) sum
      // dzG[j] * (a_j0, a_j1, 1) into sample j's slot
      if (h == 0) {
        const int p = w * 32 + r, m = swap23(p);
        const float d = Gb[j * kH + p];
        float* acc2 = L.aeacc + j * kH + m;
        acc2[0] += d * in[IL::kAct + 2 * j];
        acc2[2 * kH] += d * in[IL::kAct + 2 * j + 1];
        acc2[4 * kH] += d;
      }
      // dW2[own][2j, 2j+1] += dz2^T h1g (after L3: its fragments and h1 are dead by now)
      const TrA<kH> TA = tr_base<kH, true>(LB, lane);
      mfma_grid<G / 16, 2>([&](int kk) { return trf(L.b, TA, kk, w); },
                           [&](int kk, int n) { return trf(L.a, TA, kk, 2 * j + n); },
                           [&](int kk, int n, const frag8& A, const frag8& B) {
                             if (n == 0 && j == 0) db2 += sum8(A);
                             mfma_acc(dW2[n], A, B);
                           });
    }
#pragma unroll
    for (int u = 0; u < kPer8; ++u) {
      const int e = tid_p + u * kT8;
      if (e < IL::kSize) L.in[buf ^ 1][e] = pre[u];
    }
    __syncthreads();

    frag8 wt[8];
    // ---------------- dW1[own][4j .. 4j+3] += dz1^T x; the next round's images staged; L4: dx = W1^T dz1 for cos
    // block cb, c recomputed -> dF, dzc; the encoders' sums; dWc[cb] += dzc^T cos
    {
      ASVRL_FRESH_LANE();
      const int v = __builtin_amdgcn_readfirstlane(tid_ >> 6);
      const int w = v & 3, j = v >> 2;
      const TrA<kH> TA_d = tr_base<kH, true>(LB, lane);
      const TrA<kC> TA_x = tr_base<kC, true>(LB, lane);
      mfma_grid<G / 16, 4>([&](int kk) { return trf(L.dz1, TA_d, kk, w); },
                           [&](int kk, int n) { return trf(L.x, TA_x, kk, 4 * j + n); },
                           [&](int kk, int n, const frag8& A, const frag8& B) {
                             if (n == 0 && j == 0) db1 += sum8(A);
                             mfma_acc(dW1[n], A, B);
                           });
      // L4's W1^T fragments for cos block cb, in flight while the next round's images are staged
      const frag8* W1T = reinterpret_cast<const frag8*>(a.w.w1t_frag);
#pragma unroll
      for (int ks = 0; ks < 8; ++ks) wt[ks] = W1T[((2 * w + j) * 8 + ks) * 64 + lane];
    }
    __builtin_amdgcn_sched_barrier(0);
    {
      const int tn = t + static_cast<int>(gridDim.x);
      if (tn < a.rounds) stage(L.in[buf ^ 1], L.cos[buf ^ 1], L.F[buf ^ 1], L.G[buf ^ 1], false);
    }
    __builtin_amdgcn_sched_barrier(0);
    {
      ASVRL_FRESH_LANE();
      const int v = __builtin_amdgcn_readfirstlane(tid_ >> 6);
      const int w = v & 3, j = v >> 2, cb = 2 * w + j;
      {   // cos block cb's Wc fragments: first used after the 16 dx MFMAs below
        const frag8* WC = reinterpret_cast<const frag8*>(a.w.wc_frag);
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) wcr[ks] = WC[(cb * 4 + ks) * 64 + lane];
      }
      const RowA<kNcos> RA_cos = row_base<kNcos, true>(LB, lane, r, h);
      const RowA<kH> RA_d = row_base<kH, true>(LB, lane, r, h);
      elem_t* const dzc_w = L.dzc[w];
      // dx of both row blocks first (the W1^T fragments then die), then per row block c and the epilogue
      f32x16 dxs[NB];
#pragma unroll
      for (int rb = 0; rb < NB; ++rb) dxs[rb] = f32x16{};
      mfma_rows<8, NB>(dxs, L.dz1, RA_d, [&](int ks) { return wt[ks]; });
#pragma unroll
      for (int rb = 0; rb < NB; ++rb) {
        f32x16 cc[1] = {acc_init(bcp, cb * 32, h)};
        mfma_rows<4, 1>(cc, cosb + rb * 32 * kNcos, RA_cos, [&](int ks) { return wcr[ks]; });
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          float fv[8], cv[8], d[8], fs[8], df[8], dz[8];
          lds8(Fb + rb * kC + cb * 32 + 16 * s + 8 * h, fv);
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            cv[i] = relu(cc[0][8 * s + i]);
            d[i] = dxs[rb][8 * s + i];
          }
          mul8(d, cv, fs);
          mul8(d, fv, df);
#pragma unroll
          for (int i = 0; i < 8; ++i) dz[i] = cv[i] > 0.f ? df[i] : 0.f;
          rows(dzc_w, RA_cos, rb, 2 * j + s, pack8(dz));   // dzc = dx F 1[c > 0], this wave's half of image w
          // dF of sample rb = sum over its taus of dx c -> dzF = dF 1[F > 0], in place over F's block cb (the
          // positions this wave's half h holds: 16 s + 8 h + i)
          half_rows_sum8(fs, lane);
          if (r < 8) {
            const int p = cb * 32 + 16 * s + 8 * h + r;
            const float fm = Fb[rb * kC + p];
            Fb[rb * kC + p] = fm > 0.f ? fs[0] : 0.f;
          }
        }
      }
      // the observation encoders' gradients (AC_IQN_model.py:284-308): lane (h, r) takes feature
      // m = swap23(32 cb + r) of sample h; the two samples' sums added in sample order (half_sum)
      {
        const int p = cb * 32 + r, m = swap23(p);
        const bool self = m < kSelfF;
        const int off = self ? 0 : kSelfIn + kObjIn * ((m - kSelfF) / kObjF);
        const float d = Fb[h * kC + p];
        const float* x = in + IL::kObs + h * kObsIn + off;
        float e8[8];
#pragma unroll
        for (int i = 0; i < kSelfIn; ++i) e8[i] = half_sum(d * ((self || i < kObjIn) ? x[i] : 0.f));
        e8[7] = half_sum(d);
        if (h == 0)
#pragma unroll
          for (int i = 0; i < 8; ++i) L.encacc[i * kC + m] += e8[i];
      }
      const TrA<kNcos> TA_c = tr_base<kNcos, true>(LB, lane);
#pragma unroll
      for (int kk = 0; kk < G / 16; ++kk) {
        const frag8 A = trf(dzc_w, TA_c, kk, j);
        dbc += sum8(A);
#pragma unroll
        for (int n = 0; n < 2; ++n) mfma_acc(dWc[n], A, trf(cosb, TA_c, kk, n));
      }
      // the next round's L0 fragments (the same Wc; not held through L1 .. L3)
      const frag8* WC = reinterpret_cast<const frag8*>(a.w.wc_frag);
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) wcr[ks] = WC[(cb * 4 + ks) * 64 + lane];
    }
    __syncthreads();   // the next round overwrites x, a, b, dz1, the exchange slots and dzc
  }

  // ---------------- the workgroup's partials
  mfma_drain();
  const int lane = threadIdx.x & 63, v = threadIdx.x >> 6, w = v & 3, j = v >> 2, h = lane >> 5, r = lane & 31;
  const int grp = blockIdx.x;
  if (a.parts.enc != nullptr) {
    const float* ea = L.encacc;
    float* pe = a.parts.enc + static_cast<size_t>(grp) * 688;
    for (int i = threadIdx.x; i < 688; i += kT8) {
      float val;
      if (i < kSelfF * kSelfIn) val = ea[(i % kSelfIn) * kC + i / kSelfIn];
      else if (i < kSelfF * (kSelfIn + 1)) val = ea[7 * kC + i - kSelfF * kSelfIn];
      else {
        const int e = i - kSelfF * (kSelfIn + 1);
        const int jf = e < kObjF * kObjIn ? e / kObjIn : e - kObjF * kObjIn;
        const int slot = e < kObjF * kObjIn ? e % kObjIn : 7;
        val = 0.f;
#pragma unroll
        for (int o = 0; o < 5; ++o) val += ea[slot * kC + kSelfF + kObjF * o + jf];
      }
      pe[i] = val;
    }
  }
  if (a.parts.aenc != nullptr) {
    float* pa = a.parts.aenc + static_cast<size_t>(grp) * (3 * kH);
    for (int i = threadIdx.x; i < 3 * kH; i += kT8) {
      const int m = i < 2 * kH ? i / 2 : i - 2 * kH, c = i < 2 * kH ? i % 2 : 2;
      pa[i] = L.aeacc[(2 * c) * kH + m] + L.aeacc[(2 * c + 1) * kH + m];
    }
  }
  float* p2 = a.parts.hidden2 + static_cast<size_t>(grp) * (kH * kH + kH);
  float* p1 = a.parts.hidden + static_cast<size_t>(grp) * (kH * kC + kH);
  float* pc = a.parts.cos_emb + static_cast<size_t>(grp) * (kC * kNcos + kC);
  const int cb = 2 * w + j;
#pragma unroll
  for (int g = 0; g < 16; ++g) {
    const int m = (g & 3) + 8 * (g >> 2) + 4 * h;   // MFMA C row of register g
    const int f2 = swap23(w * 32 + m);
#pragma unroll
    for (int n = 0; n < 2; ++n) p2[f2 * kH + swap23(32 * (2 * j + n) + r)] = dW2[n][g];
#pragma unroll
    for (int n = 0; n < 4; ++n) p1[f2 * kC + swap23(32 * (4 * j + n) + r)] = dW1[n][g];
    const int fc = swap23(cb * 32 + m);
#pragma unroll
    for (int n = 0; n < 2; ++n) pc[fc * kNcos + 32 * n + r] = dWc[n][g];
  }
  dbc = half_sum(dbc);
  db2 = half_sum(db2);
  db1 = half_sum(db1);
  if (h == 0) {
    if (j == 0) {
      p2[kH * kH + swap23(w * 32 + r)] = db2;
      p1[kH * kC + swap23(w * 32 + r)] = db1;
    }
    pc[kC * kNcos + swap23(cb * 32 + r)] = dbc;
  }
  // the output layer: each half's row sums per feature position, then the two halves in order; bo from waves 0-3
  if (r < 16) red8[j][w * 32 + 16 * (r >> 3) + 8 * h + (r & 7)] = dwo1;
  dbo = seg_sum<32>(h == 0 ? dbo : 0.f);
  if (lane == 31 && v < 4) L.red[v] = dbo;
  __syncthreads();
  float* po = a.parts.out + static_cast<size_t>(grp) * (kH + 1);
  if (threadIdx.x < kH) po[swap23(threadIdx.x)] = red8[0][threadIdx.x] + red8[1][threadIdx.x];
  if (threadIdx.x == 0) po[kH] = ((L.red[0] + L.red[1]) + L.red[2]) + L.red[3];
}
#endif  // !ASVRL_OPERAND_F32

int fused_nb(int N) {
#if ASVRL_OPERAND_F32
  (void)N;
  return 1;
#else
  return 2;
#endif
}

int fused_rounds(int B, int N) { return static_cast<int>(static_cast<int64_t>(B) * N / (32 * fused_nb(N))); }

}  // namespace
}  // namespace asvrl

using namespace asvrl;


#ifdef ASVRL_FUSED_STAMPS
extern "C" int asvrl_debug_fused_stamps(uint64_t* out, int64_t n) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps), n * sizeof(uint64_t)) == hipSuccess ? 0 : 1;
}
#endif

// one workgroup per CU (leaving CUs to the concurrent rollout stream measured slower, profiles/r02_cu_reserve_ab.txt)
extern "C" int32_t asvrl_critic_fused_groups(int32_t B, int32_t N) {
  if (B <= 0 || (N != 8 && N != 16 && N != 32)) return 0;
  const int rounds = fused_rounds(B, N);
  const int cus = cu_count();
  return rounds < cus ? rounds : cus;
}

namespace {
// which kernel asvrl_critic_train_fused(_tq) launches where both take the shape: 4 (default) critic_fused_kernel,
// 8 critic_fused8_kernel (asvrl_critic_fused_variant; measured 11 % slower, kept for the A/B and its tests)
int g_fused_variant = 4;

int critic_train_fused_launch(const AsvCriticWeights* w, const AsvCriticIO* io, const AsvCriticParts* parts,
                              const AsvCriticWeights* tw, const AsvCriticIO* tio, void* stream) {
  ASVRL_REQUIRE(w && io && parts, "asvrl_critic_train_fused: null argument");
  ASVRL_REQUIRE(io->taus && io->obs && io->act && io->q_next && io->rewards && io->dones,
                "asvrl_critic_train_fused: needs taus, obs, act, q_next, rewards and dones");
  ASVRL_REQUIRE(io->ld_obs >= 37, "asvrl_critic_train_fused: ld_obs must cover the packed observation row");
  ASVRL_REQUIRE(w->wc_frag && w->w1_frag && w->w2_frag && w->w2t_frag && w->w1t_frag && w->bc && w->b1 && w->b2 &&
                    w->wo && w->bo && w->self_w && w->self_b && w->obj_w && w->obj_b && w->ae_w && w->ae_b,
                "asvrl_critic_train_fused: null weight");
  ASVRL_REQUIRE(parts->cos_emb && parts->hidden && parts->hidden2 && parts->out,
                "asvrl_critic_train_fused: null partial buffer");
  ASVRL_REQUIRE(io->N == 8 || io->N == 16 || io->N == 32, "asvrl_critic_train_fused: N must be 8, 16 or 32");
  ASVRL_REQUIRE(io->Np == io->N, "asvrl_critic_train_fused: N' must equal N");
  ASVRL_REQUIRE(io->kappa > 0.f, "asvrl_critic_train_fused: kappa must be positive");
  ASVRL_REQUIRE(io->B >= 0 && (static_cast<int64_t>(io->B) * io->N) % (32 * fused_nb(io->N)) == 0,
                "asvrl_critic_train_fused: B*N must be a multiple of the round size (64 rows; 32 in the f32 build)");
  const bool tq = tw != nullptr;
  if (tq) {
    ASVRL_REQUIRE(tio != nullptr, "asvrl_critic_train_fused_tq: null target IO");
    ASVRL_REQUIRE(tw->wc_frag && tw->w1_frag && tw->w2_frag && tw->bc && tw->b1 && tw->b2 && tw->wo && tw->bo &&
                      tw->self_w && tw->self_b && tw->obj_w && tw->obj_b && tw->ae_w && tw->ae_b,
                  "asvrl_critic_train_fused_tq: null target weight");
    ASVRL_REQUIRE(tio->taus && tio->obs && tio->act, "asvrl_critic_train_fused_tq: the target pass needs taus, obs and act");
    ASVRL_REQUIRE(tio->ld_obs >= 37, "asvrl_critic_train_fused_tq: target ld_obs must cover the packed observation row");
    ASVRL_REQUIRE(tio->B == io->B && tio->N == io->N, "asvrl_critic_train_fused_tq: target B / N differ from the update's");
  }
  if (io->B == 0) return 0;
  FusedArgs a{};
  a.w = *w;
  a.obs = io->obs; a.ld_obs = io->ld_obs; a.ain = io->act; a.ld_ain = io->ld_act; a.xb = io->xb;
  a.taus = io->taus; a.qn = io->q_next; a.rew = io->rewards; a.don = io->dones; a.ld_rd = io->ld_rd;
  a.gamma = io->gamma; a.kappa = io->kappa;
  a.gscale = 1.f / (static_cast<float>(io->B) * static_cast<float>(io->Np));
  a.loss_scale = io->loss_scale;
  a.B = io->B;
  a.rounds = fused_rounds(io->B, io->N);
  a.q = io->q; a.row_loss = io->row_loss; a.tile_loss = io->tile_loss;
  a.dzF = io->dzF; a.dzG = io->dzG;
  a.parts = *parts;
  if (tq) {
    a.tq = ctile::make_args(tw, tio);
    a.tq.F = nullptr;
    a.tq.G = nullptr;
    a.tq.q = const_cast<float*>(io->q_next);   // written here, read by the rounds
  }
  const int grid = asvrl_critic_fused_groups(io->B, io->N);
  hipStream_t st = as_stream(stream);
#if !ASVRL_OPERAND_F32
  // the two-waves-per-SIMD kernel wherever it takes the shape (AC-IQN N = 32, encoders in the launch)
  if (g_fused_variant == 8 && io->N == 32 && parts->enc != nullptr && parts->aenc != nullptr && io->dzF == nullptr &&
      io->dzG == nullptr && io->xb == nullptr) {
    if (tq) hipLaunchKernelGGL((critic_fused8_kernel<true>), dim3(grid), dim3(kT8), 0, st, a);
    else hipLaunchKernelGGL((critic_fused8_kernel<false>), dim3(grid), dim3(kT8), 0, st, a);
    return check_launch(tq ? "asvrl_critic_train_fused_tq" : "asvrl_critic_train_fused");
  }
#endif
  if (tq) {
    if (io->N == 32) hipLaunchKernelGGL((critic_fused_kernel<32, false, true>), dim3(grid), dim3(kNW * 64), 0, st, a);
    else if (io->N == 16) hipLaunchKernelGGL((critic_fused_kernel<16, false, true>), dim3(grid), dim3(kNW * 64), 0, st, a);
    else hipLaunchKernelGGL((critic_fused_kernel<8, false, true>), dim3(grid), dim3(kNW * 64), 0, st, a);
    return check_launch("asvrl_critic_train_fused_tq");
  }
  if (io->N == 32) hipLaunchKernelGGL((critic_fused_kernel<32, false>), dim3(grid), dim3(kNW * 64), 0, st, a);
  else if (io->N == 16) hipLaunchKernelGGL((critic_fused_kernel<16, false>), dim3(grid), dim3(kNW * 64), 0, st, a);
  else hipLaunchKernelGGL((critic_fused_kernel<8, false>), dim3(grid), dim3(kNW * 64), 0, st, a);
  return check_launch("asvrl_critic_train_fused");
}
}  // namespace

extern "C" int asvrl_critic_train_fused(const AsvCriticWeights* w, const AsvCriticIO* io, const AsvCriticParts* parts,
                                        void* stream) {
  return critic_train_fused_launch(w, io, parts, nullptr, nullptr, stream);
}

extern "C" int asvrl_critic_train_fused_tq(const AsvCriticWeights* w, const AsvCriticIO* io, const AsvCriticParts* parts,
                                           const AsvCriticWeights* tw, const AsvCriticIO* tio, void* stream) {
  ASVRL_REQUIRE(tw != nullptr, "asvrl_critic_train_fused_tq: null target weights");
  return critic_train_fused_launch(w, io, parts, tw, tio, stream);
}

// train_IQN's update (agent.py:449-468) in one launch: the same kernel with IQN_Policy's trunk (no action
// encoder, IQN_model.py:74-108) and its 128 -> A output layer gathered at the taken action; the output
// layer's partial is [32 x 128 + 32] per workgroup (rows >= n_actions zero). With tw (asvrl_iqn_train_fused_tq,
// ABI 24) the target network's max over the actions (agent.py:451-452) is computed inside the launch first.
namespace {
int iqn_train_fused_launch(const AsvCriticWeights* w, const AsvIqnHead* head, const AsvIqnIO* io,
                           const AsvCriticParts* parts, const AsvCriticWeights* tw, const AsvIqnHead* thead,
                           const AsvIqnIO* tio, void* stream) {
  ASVRL_REQUIRE(w && head && io && parts, "asvrl_iqn_train_fused: null argument");
  ASVRL_REQUIRE(io->taus && io->obs && io->actions && io->q_next && io->rewards && io->dones,
                "asvrl_iqn_train_fused: needs taus, obs, actions, q_next, rewards and dones");
  ASVRL_REQUIRE(io->ld_obs >= 37, "asvrl_iqn_train_fused: ld_obs must cover the packed observation row");
  ASVRL_REQUIRE(w->wc_frag && w->w1_frag && w->w2_frag && w->w2t_frag && w->w1t_frag && w->bc && w->b1 && w->b2 &&
                    w->self_w && w->self_b && w->obj_w && w->obj_b,
                "asvrl_iqn_train_fused: null weight");
  ASVRL_REQUIRE(head->wo && head->bo && head->n_actions >= 1 && head->n_actions <= kMaxA,
                "asvrl_iqn_train_fused: bad head");
  ASVRL_REQUIRE(parts->cos_emb && parts->hidden && parts->hidden2 && parts->out,
                "asvrl_iqn_train_fused: null partial buffer");
  ASVRL_REQUIRE(parts->aenc == nullptr, "asvrl_iqn_train_fused: IQN_Policy has no action encoder (parts->aenc)");
  ASVRL_REQUIRE(io->N == 8 || io->N == 16 || io->N == 32, "asvrl_iqn_train_fused: N must be 8, 16 or 32");
  ASVRL_REQUIRE(io->Np == io->N, "asvrl_iqn_train_fused: N' must equal N");
  ASVRL_REQUIRE(io->kappa > 0.f, "asvrl_iqn_train_fused: kappa must be positive");
  ASVRL_REQUIRE(io->B >= 0 && (static_cast<int64_t>(io->B) * io->N) % (32 * fused_nb(io->N)) == 0,
                "asvrl_iqn_train_fused: B*N must be a multiple of the round size (64 rows; 32 in the f32 build)");
  const bool tq = tw != nullptr;
  if (tq) {
    ASVRL_REQUIRE(thead && tio, "asvrl_iqn_train_fused_tq: null target head or IO");
    ASVRL_REQUIRE(tw->wc_frag && tw->w1_frag && tw->w2_frag && tw->bc && tw->b1 && tw->b2 && tw->self_w &&
                      tw->self_b && tw->obj_w && tw->obj_b,
                  "asvrl_iqn_train_fused_tq: null target weight");
    ASVRL_REQUIRE(thead->wo_frag && thead->bo && thead->n_actions == head->n_actions,
                  "asvrl_iqn_train_fused_tq: bad target head");
    ASVRL_REQUIRE(tio->taus && tio->obs && tio->ld_obs >= 37,
                  "asvrl_iqn_train_fused_tq: the target pass needs taus and obs (packed observation rows)");
    ASVRL_REQUIRE(tio->B == io->B && tio->N == io->N, "asvrl_iqn_train_fused_tq: target B / N differ from the update's");
  }
  if (io->B == 0) return 0;
  FusedArgs a{};
  a.w = *w;
  a.obs = io->obs; a.ld_obs = io->ld_obs; a.ain = io->actions; a.ld_ain = io->ld_rd; a.xb = io->xb;
  a.taus = io->taus; a.qn = io->q_next; a.rew = io->rewards; a.don = io->dones; a.ld_rd = io->ld_rd;
  a.gamma = io->gamma; a.kappa = io->kappa;
  a.gscale = 1.f / (static_cast<float>(io->B) * static_cast<float>(io->Np));
  a.loss_scale = io->loss_scale;
  a.B = io->B;
  a.rounds = fused_rounds(io->B, io->N);
  a.q = io->q; a.row_loss = io->row_loss; a.tile_loss = io->tile_loss;
  a.dzF = io->dzF; a.dzG = nullptr;
  a.parts = *parts;
  a.iwo = head->wo; a.ibo = head->bo; a.n_actions = head->n_actions;
  if (tq) {   // asvrl_iqn_forward_max's arguments (asvrl_critic.hip iqn_args), q -> the update's q_next
    a.tq.w = *tw;
    a.tq.hd = *thead;
    a.tq.taus = tio->taus; a.tq.B = tio->B; a.tq.N = tio->N; a.tq.Np = tio->N;
    a.tq.obs = tio->obs; a.tq.ld_obs = tio->ld_obs;
    a.tq.q = const_cast<float*>(io->q_next);   // written here, read by the rounds
  }
  const int grid = asvrl_critic_fused_groups(io->B, io->N);
  hipStream_t st = as_stream(stream);
  if (tq) {
    if (io->N == 32) hipLaunchKernelGGL((critic_fused_kernel<32, true, true>), dim3(grid), dim3(kNW * 64), 0, st, a);
    else if (io->N == 16) hipLaunchKernelGGL((critic_fused_kernel<16, true, true>), dim3(grid), dim3(kNW * 64), 0, st, a);
    else hipLaunchKernelGGL((critic_fused_kernel<8, true, true>), dim3(grid), dim3(kNW * 64), 0, st, a);
    return check_launch("asvrl_iqn_train_fused_tq");
  }
  if (io->N == 32) hipLaunchKernelGGL((critic_fused_kernel<32, true>), dim3(grid), dim3(kNW * 64), 0, st, a);
  else if (io->N == 16) hipLaunchKernelGGL((critic_fused_kernel<16, true>), dim3(grid), dim3(kNW * 64), 0, st, a);
  else hipLaunchKernelGGL((critic_fused_kernel<8, true>), dim3(grid), dim3(kNW * 64), 0, st, a);
  return check_launch("asvrl_iqn_train_fused");
}
}  // namespace

extern "C" int asvrl_iqn_train_fused(const AsvCriticWeights* w, const AsvIqnHead* head, const AsvIqnIO* io,
                                     const AsvCriticParts* parts, void* stream) {
  return iqn_train_fused_launch(w, head, io, parts, nullptr, nullptr, nullptr, stream);
}

extern "C" int asvrl_iqn_train_fused_tq(const AsvCriticWeights* w, const AsvIqnHead* head, const AsvIqnIO* io,
                                        const AsvCriticParts* parts, const AsvCriticWeights* tw,
                                        const AsvIqnHead* thead, const AsvIqnIO* tio, void* stream) {
  ASVRL_REQUIRE(tw != nullptr, "asvrl_iqn_train_fused_tq: null target weights");
  return iqn_train_fused_launch(w, head, io, parts, tw, thead, tio, stream);
}

// The AC-IQN critic update's kernel where both forms take the shape (N = 32, encoders' gradients in the launch,
// bf16 build): 4 = critic_fused_kernel (one wave per SIMD, the default), 8 = critic_fused8_kernel (two waves per
// SIMD). v < 0 only queries. Returns the previous setting; anything else is an error (-1).
extern "C" int32_t asvrl_critic_fused_variant(int32_t v) {
  const int prev = g_fused_variant;
  if (v < 0) return prev;
  if (v != 4 && v != 8) {
    set_error("asvrl_critic_fused_variant: variant must be 4 or 8");
    return -1;
  }
  g_fused_variant = v;
  return prev;
}
