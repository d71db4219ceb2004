// asvrl_mlp.hip -- the per-row MLPs of AC-IQN on MFMA (gfx950): the observation encoders
// (AC_IQN_model.py:284-308: self_encoder 7 -> 56, object_encoder 5 -> 40 per object, masked,
// concatenated to 256), the Actor head (:310-321: 256 -> 128 -> 128 -> 2, (2/pi) atan) and the
// critic's action_encoder (2 -> 128).
//
// The two encoders are ONE block-structured 256 x 32 matrix acting on columns 0..31 of the packed
// observation row [self 7 | objects 5x5 | mask 5 | pad 3]: rows 0..55 see columns 0..6 (self),
// rows 56+40o .. 95+40o see columns 7+5o .. 11+5o (object o). masked_fill(mask < 0.5, 0) is a
// per-feature multiplier in the epilogue. Same tile convention as the critic (asvrl_mfma.h):
// one wave = 32 rows, features on the MFMA M dimension, accumulators chained as B operands.
//
// Kernels:
//   encode_kernel          F = encoders(obs) [B][256] f32 and G = relu(W_ae a + b_ae) [B][128] f32, plus a
//                          bf16 copy of obs columns 0..31 (operand of the encoder wgrad)
//   actor_kernel<ACT>      Actor on every robot row with epsilon-greedy exploration (agent.py:207-225,
//                          trainer.py:257-264): f64 actions for the env kernel; one wave per 32-row
//                          tile, weights staged in LDS
//   actor_split_kernel     the learner's B rows, 4 waves per tile splitting each layer's features:
//     <FWD>                f32 actions (target actor, agent.py:398)
//     <TRAIN>              saving bf16 activations for the backward (agent.py:419-426)
//   actor_bwd_split_kernel the actor backward from dL/d(action) to the encoders' pre-activations
#include "asvrl_common.h"
#include "asvrl_mfma.h"
#include "asvrl_lds.h"

namespace asvrl {
namespace {

// The split actor kernels run one wave per SIMD (4 waves per 32-row workgroup), so a weight fragment
// fetched from L2 right before its MFMA exposes the whole L2 latency on every MFMA of a chain. With
// ASVRL_MLP_WPRE a chain's fragments are all fetched first (A/B knob; same MFMA order, bit-identical).
#ifndef ASVRL_MLP_WPRE
#define ASVRL_MLP_WPRE 0
#endif
template <int KS, int P>
__device__ __forceinline__ f32x16 wchain(const frag8* W, int base, int lane, const elem_t* img, const RowA<P>& RA) {
  f32x16 acc = f32x16{};
  if constexpr (ASVRL_MLP_WPRE != 0) {
    frag8 q[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) q[ks] = W[(base + ks) * 64 + lane];
    if constexpr (ASVRL_MLP_WPRE >= 2) {   // the LDS operands too
      frag8 b[KS];
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) b[ks] = rowf(img, RA, 0, ks);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) acc = mfma(q[ks], b[ks], acc);
    } else {
      __builtin_amdgcn_sched_barrier(0);   // every fetch issued before the chain (not sunk to its MFMA)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) acc = mfma(q[ks], rowf(img, RA, 0, ks), acc);
    }
  } else {
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) acc = mfma(W[(base + ks) * 64 + lane], rowf(img, RA, 0, ks), acc);
  }
  return acc;
}

constexpr int kEnc = 256, kObsK = 32, kHid = 128, kNa = 2;
constexpr int kSelfF = 56, kObjF = 40, kSelfIn = 7, kObjIn = 5, kObjN = 5;
constexpr int kFragEnc = kEnc * kObsK / 8;   // 1024 fragments
constexpr int kFragAe = kHid * 16 / 8;       // 256 (action encoder, K padded 2 -> 16)
constexpr int kFragH1 = kHid * kEnc / 8;     // 4096
constexpr int kFragH2 = kHid * kHid / 8;     // 2048
constexpr int kMlpWaves = 4;

enum { MLP_ENCODE = 0, MLP_ACT = 1, MLP_FWD = 2, MLP_TRAIN = 3 };

struct MlpArgs {
  AsvMlpWeights w;
  AsvMlpIO io;
};

struct ActorLds {
  frag8 enc[lds_frags(kFragEnc)];
  frag8 w1[lds_frags(kFragH1)];
  frag8 w2[lds_frags(kFragH2)];
  float benc[kEnc], b1[kHid], b2[kHid], wout[kNa * kHid], bout[kNa];
};

// object index of encoder feature m (>= 56)
__host__ __device__ constexpr int obj_of(int m) { return (m - kSelfF) / kObjF; }

// Encoder output of one 32-row tile: B operand from obs columns 0..31, 8 blocks in 2 halves;
// epilogue bias + relu + mask. Hands each finished (block, s) group of 8 features to `emit`.
template <typename Emit>
__device__ __forceinline__ void encode_tile(const frag8* ENC, const float* benc, const frag8 (&bx)[2],
                                            const float (&mk)[kObjN], int lane, Emit emit) {
  const int h = lane >> 5;
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    f32x16 acc[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[q] = f32x16{};
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[q] = mfma(ENC[((half * 4 + q) * 2 + ks) * 64 + lane], bx[ks], acc[q]);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int mb = half * 4 + q;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int g = 8 * s + j;
          const int m0 = mb * 32 + (g & 3) + 8 * (g >> 2);   // feature for h = 0; h = 1 adds 4
          const float mk0 = m0 < kSelfF ? 1.f : (mk[obj_of(m0)] < 0.5f ? 0.f : 1.f);
          const float mk1 = m0 + 4 < kSelfF ? 1.f : (mk[obj_of(m0 + 4)] < 0.5f ? 0.f : 1.f);
          float x = acc[q][g] + benc[m0 + 4 * h];
          x = relu(x);
          v[j] = x * (h ? mk1 : mk0);
        }
        emit(mb, s, v);
      }
    }
  }
}

// bf16 B operand of the encoder (obs columns 0..31) + the object mask, for row `row`
__device__ __forceinline__ void load_obs(const float* __restrict__ x, int64_t ldx, int row, int h, frag8 (&bx)[2],
                                         float (&mk)[kObjN]) {
  const float* xr = x + static_cast<int64_t>(row) * ldx;
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    const float4 u = *reinterpret_cast<const float4*>(xr + ks * 16 + 8 * h);
    const float4 v = *reinterpret_cast<const float4*>(xr + ks * 16 + 8 * h + 4);
    const float e[8] = {u.x, u.y, u.z, u.w, v.x, v.y, v.z, v.w};
    bx[ks] = pack8(e);
  }
#pragma unroll
  for (int o = 0; o < kObjN; ++o) mk[o] = xr[32 + o];
}

// ------------------------------------------------------------------ ENCODE (critic F, G)
__global__ __launch_bounds__(kMlpWaves * 64) void encode_kernel(MlpArgs a) {
  const int lane = threadIdx.x & 63, h = lane >> 5, r = lane & 31;
  const int tile = blockIdx.x * kMlpWaves + (threadIdx.x >> 6);
  const AsvMlpIO& io = a.io;
  if (tile * 32 >= io.n) return;
  const int row = tile * 32 + r;
  const bool valid = row < io.n;
  const int rr = valid ? row : io.n - 1;
  frag8 bx[2];
  float mk[kObjN];
  load_obs(io.x, io.ldx, rr, h, bx, mk);
  if (io.xb != nullptr && valid) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
      *reinterpret_cast<frag8*>(bp(io.xb) + static_cast<int64_t>(row) * kObsK + ks * 16 + 8 * h) = bx[ks];
  }
  const frag8* ENC = reinterpret_cast<const frag8*>(a.w.enc_frag);
  float* Fr = io.F + static_cast<int64_t>(rr) * kEnc;
  encode_tile(ENC, a.w.b_enc, bx, mk, lane, [&](int mb, int s, const float* v) {
    if (!valid) return;
    float* o = Fr + mb * 32 + 16 * s + 4 * h;
    *reinterpret_cast<float4*>(o) = make_float4(v[0], v[1], v[2], v[3]);
    *reinterpret_cast<float4*>(o + 8) = make_float4(v[4], v[5], v[6], v[7]);
  });
  if (io.G == nullptr) return;
  // action encoder: B operand = (a0, a1, 0, ...) in lane half 0
  frag8 ba{};
  if (h == 0) {
    const float* ar = io.act + static_cast<int64_t>(rr) * io.lda;
    ba[0] = (elem_t)ar[0];
    ba[1] = (elem_t)ar[1];
  }
  const frag8* AE = reinterpret_cast<const frag8*>(a.w.ae_frag);
  float* Gr = io.G + static_cast<int64_t>(rr) * kHid;
#pragma unroll
  for (int mb = 0; mb < 4; ++mb) {
    const f32x16 acc = mfma(AE[mb * 64 + lane], ba, f32x16{});
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float x = acc[8 * s + j] + a.w.b_ae[feat(mb, 8 * s + j, h)];
        v[j] = relu(x);
      }
      if (valid) {
        float* o = Gr + mb * 32 + 16 * s + 4 * h;
        *reinterpret_cast<float4*>(o) = make_float4(v[0], v[1], v[2], v[3]);
        *reinterpret_cast<float4*>(o + 8) = make_float4(v[4], v[5], v[6], v[7]);
      }
    }
  }
}

// ------------------------------------------------------------------ Actor forward (ACT/FWD/TRAIN)
template <int MODE>
__device__ __forceinline__ void actor_tile(const MlpArgs& a, const ActorLds& L, int tile, int lane,
                                           const frag8 (&bx)[2], const float (&mk)[kObjN]) {
  const AsvMlpIO& io = a.io;
  const int h = lane >> 5, r = lane & 31;
  const int row = tile * 32 + r;
  const bool valid = row < io.n;
  if (MODE == MLP_TRAIN && valid) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
      *reinterpret_cast<frag8*>(bp(io.xb) + static_cast<int64_t>(row) * kObsK + ks * 16 + 8 * h) = bx[ks];
  }
  // encoders -> h0 (chained B operand of hidden_layer)
  frag8 fpk[16];
  encode_tile(wimg(L.enc, a.w.enc_frag), L.benc, bx, mk, lane, [&](int mb, int s, const float* v) {
    fpk[mb * 2 + s] = pack8(*reinterpret_cast<const float (*)[8]>(v));
    if (MODE == MLP_TRAIN)
      store16(valid ? bp(io.h0) + static_cast<int64_t>(row) * kEnc + mb * 32 + 16 * s : nullptr, v, h);
  });
  // hidden_layer 256 -> 128, relu
  const frag8* W1 = wimg(L.w1, a.w.w1_frag);
  const frag8* W2 = wimg(L.w2, a.w.w2_frag);
  f32x16 acc1[4];
#pragma unroll
  for (int mb = 0; mb < 4; ++mb) acc1[mb] = f32x16{};
#pragma unroll
  for (int ks = 0; ks < kEnc / 16; ++ks)
#pragma unroll
    for (int mb = 0; mb < 4; ++mb) acc1[mb] = mfma(W1[(mb * 16 + ks) * 64 + lane], fpk[ks], acc1[mb]);
  frag8 h1pk[8];
#pragma unroll
  for (int mb = 0; mb < 4; ++mb)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float x = acc1[mb][8 * s + j] + L.b1[feat(mb, 8 * s + j, h)];
        v[j] = relu(x);
      }
      h1pk[mb * 2 + s] = pack8(v);
      if (MODE == MLP_TRAIN)
      store16(valid ? bp(io.h1) + static_cast<int64_t>(row) * kHid + mb * 32 + 16 * s : nullptr, v, h);
    }
  // hidden_layer_2 128 -> 128, relu; output_layer 128 -> 2
  f32x16 acc2[4];
#pragma unroll
  for (int mb = 0; mb < 4; ++mb) acc2[mb] = f32x16{};
#pragma unroll
  for (int ks = 0; ks < kHid / 16; ++ks)
#pragma unroll
    for (int mb = 0; mb < 4; ++mb) acc2[mb] = mfma(W2[(mb * 8 + ks) * 64 + lane], h1pk[ks], acc2[mb]);
  float p0 = 0.f, p1 = 0.f;
#pragma unroll
  for (int mb = 0; mb < 4; ++mb)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int m = feat(mb, 8 * s + j, h);
        const float x = acc2[mb][8 * s + j] + L.b2[m];
        v[j] = relu(x);
        p0 += L.wout[m] * v[j];
        p1 += L.wout[kHid + m] * v[j];
      }
      if (MODE == MLP_TRAIN)
      store16(valid ? bp(io.h2) + static_cast<int64_t>(row) * kHid + mb * 32 + 16 * s : nullptr, v, h);
    }
  const float z0 = p0 + __shfl_xor(p0, 32, 64) + L.bout[0];
  const float z1 = p1 + __shfl_xor(p1, 32, 64) + L.bout[1];
  const float a0 = a.w.out_scale * atanf(z0);   // atan_scale * torch.atan(actions)
  const float a1 = a.w.out_scale * atanf(z1);
  if (!valid || h != 0) return;
  if (MODE == MLP_ACT) {
    // epsilon-greedy (agent.py:207-225): greedy iff random() > eps, else uniform(-1, 1) per dim;
    // eps: linear schedule of the device step counter (trainer.py:257-264)
    const uint64_t step = io.step_dev != nullptr ? static_cast<uint64_t>(*io.step_dev) : 0ull;
    const double progress = static_cast<double>(step) * io.eps_steps_per_count / io.eps_total;
    const double eps = progress < io.eps_fraction
                           ? io.eps_initial + (progress / io.eps_fraction) * (io.eps_final - io.eps_initial)
                           : io.eps_final;
    const U4 u = philox4x32_10(U4{static_cast<uint32_t>(row), static_cast<uint32_t>(step),
                                  static_cast<uint32_t>(step >> 32), 0xAC7u},
                               static_cast<uint32_t>(io.seed), static_cast<uint32_t>(io.seed >> 32));
    const double c = (static_cast<double>(u.x >> 8) + 1.0) * (1.0 / 16777216.0);   // (0, 1]
    double* o = io.a_out64 + static_cast<int64_t>(row) * 2;
    if (c > eps) {
      o[0] = a0;
      o[1] = a1;
    } else {
      o[0] = 2.0 * (static_cast<double>(u.y >> 8) * (1.0 / 16777216.0)) - 1.0;
      o[1] = 2.0 * (static_cast<double>(u.z >> 8) * (1.0 / 16777216.0)) - 1.0;
    }
  } else {
    float* o = io.a_out + static_cast<int64_t>(row) * io.ld_aout;
    o[0] = a0;
    o[1] = a1;
    if (MODE == MLP_TRAIN) {
      io.pre[static_cast<int64_t>(row) * 2] = z0;
      io.pre[static_cast<int64_t>(row) * 2 + 1] = z1;
    }
  }
}

template <int MODE>
__global__ __launch_bounds__(kMlpWaves * 64) void actor_kernel(MlpArgs a) {
  __shared__ ActorLds L;
  // the tile's observation rows are loaded first, in flight under the weight staging
  const int tile = blockIdx.x * kMlpWaves + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  const bool active = tile * 32 < a.io.n;
  frag8 bx[2];
  float mk[kObjN];
  if (active) {
    const int row = tile * 32 + (lane & 31);
    load_obs(a.io.x, a.io.ldx, row < a.io.n ? row : a.io.n - 1, lane >> 5, bx, mk);
  }
  {
    const frag8* ge = reinterpret_cast<const frag8*>(a.w.enc_frag);
    const frag8* g1 = reinterpret_cast<const frag8*>(a.w.w1_frag);
    const frag8* g2 = reinterpret_cast<const frag8*>(a.w.w2_frag);
    if constexpr (kWeightsInLds) {
      constexpr int CH = kElemBytes == 2 ? 16 : 8;   // fragments in flight per thread
      copy_frags<kMlpWaves * 64, kFragEnc, CH>(L.enc, ge, threadIdx.x);
      copy_frags<kMlpWaves * 64, kFragH1, CH>(L.w1, g1, threadIdx.x);
      copy_frags<kMlpWaves * 64, kFragH2, CH>(L.w2, g2, threadIdx.x);
    }
    for (int i = threadIdx.x; i < kEnc; i += kMlpWaves * 64) L.benc[i] = a.w.b_enc[i];
    for (int i = threadIdx.x; i < kHid; i += kMlpWaves * 64) {
      L.b1[i] = a.w.b1[i];
      L.b2[i] = a.w.b2[i];
      L.wout[i] = a.w.wout[i];
      L.wout[kHid + i] = a.w.wout[kHid + i];
    }
    if (threadIdx.x < kNa) L.bout[threadIdx.x] = a.w.bout[threadIdx.x];
  }
  __syncthreads();
  if (active) actor_tile<MODE>(a, L, tile, lane, bx, mk);
}

// ------------------------------------------------------------------ Actor, feature-split form
// FWD / TRAIN on the learner's B rows: one workgroup of 4 waves per 32-row tile; the waves split every
// layer's output features and exchange the activations through LDS in chained position order
// (asvrl_lds.h), with the weight fragments read from L2. A B-row batch then runs 4 B / 32 waves instead
// of B / 32 (AC-IQN step 0.370 -> 0.350 ms with the backward below); the rollout's 20,480-row act keeps
// the one-wave-per-tile form above, where its LDS-staged weights pay (0.356 ms with the split act).
// Phase timing (tools/prologue_stamps.py; a variant build with -DASVRL_PRO_STAMPS, never the shipped
// library): thread 0 of every workgroup records s_memrealtime (100 MHz) at its phase points, each after
// draining its outstanding memory operations so the stamp marks when the phase's data arrived.
#ifdef ASVRL_PRO_STAMPS
constexpr int kProStamps = 12;
__device__ uint64_t g_pro_stamps[2048 * kProStamps];
#define PRO_STAMP(k)                                                                              \
  do {                                                                                            \
    __builtin_amdgcn_s_waitcnt(0);                                                                \
    if (threadIdx.x == 0) g_pro_stamps[blockIdx.x * kProStamps + (k)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
extern "C" int asvrl_debug_pro_stamps(uint64_t* out, int64_t n) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_pro_stamps), n * sizeof(uint64_t)) == hipSuccess ? 0 : 1;
}
#else
#define PRO_STAMP(k) \
  do {               \
  } while (0)
#endif

// The split tile's biases and output weights in LDS (b_enc | b1 | b2 | wout[2][128] | bout), staged at the
// workgroup's start with the weight fragments instead of global reads after each layer's barrier (a small
// gain; the tile's time was instruction issue at one wave per SIMD: the encoder mask's per-element select
// chain, profiles/r03pro_prologue_stamps_{before,after}.txt).
constexpr int kSbEnc = 0, kSbB1 = kEnc, kSbB2 = kSbB1 + kHid, kSbWout = kSbB2 + kHid, kSbBout = kSbWout + 2 * kHid,
              kSplitBias = kSbBout + 2;
struct ActorSplitLds {
  elem_t x0[32 * kEnc];      // h0; the backward: dz2 image
  elem_t h1[32 * kHid];      // h1; the backward: dz1 image
  float part[kMlpWaves][32][2];
  float bias[kSplitBias];
};
static_assert(kMlpWaves * 64 == kEnc && kSplitBias <= 4 * kEnc, "split_bias_fetch: four values per thread");

// thread t's share of the bias table: entries t + 256 k (issued first, stored by split_bias_store)
__device__ __forceinline__ void split_bias_fetch(const AsvMlpWeights& wt, int t, float (&v)[4]) {
  v[0] = wt.b_enc[t];
  v[1] = t < kHid ? wt.b1[t] : wt.b2[t - kHid];
  v[2] = wt.wout[t];
  v[3] = t < 2 ? wt.bout[t] : 0.f;
}

__device__ __forceinline__ void split_bias_store(ActorSplitLds& L, int t, const float (&v)[4]) {
#pragma unroll
  for (int k = 0; k < 3; ++k) L.bias[t + kEnc * k] = v[k];
  if (t < 2) L.bias[kSbBout + t] = v[3];
}

// A wave's weight fragments of the split tile (encoder blocks 2w, 2w + 1; W1 and W2 block w), fetched
// ahead by the fused prologue so that their L2 latency overlaps its replay draw.
struct SplitPre {
  frag8 enc[4];
  frag8 w1[kEnc / 16];
  frag8 w2[kHid / 16];
};

__device__ __forceinline__ void split_prefetch(const AsvMlpWeights& wt, int w, int lane, SplitPre& q) {
  const frag8* ENC = reinterpret_cast<const frag8*>(wt.enc_frag);
  const frag8* W1 = reinterpret_cast<const frag8*>(wt.w1_frag);
  const frag8* W2 = reinterpret_cast<const frag8*>(wt.w2_frag);
#pragma unroll
  for (int i = 0; i < 4; ++i) q.enc[i] = ENC[((2 * w + (i >> 1)) * 2 + (i & 1)) * 64 + lane];
#pragma unroll
  for (int ks = 0; ks < kEnc / 16; ++ks) q.w1[ks] = W1[(w * 16 + ks) * 64 + lane];
#pragma unroll
  for (int ks = 0; ks < kHid / 16; ++ks) q.w2[ks] = W2[(w * 8 + ks) * 64 + lane];
}

// One 32-row tile of the split Actor (4 waves): rows tile * 32 + r of the outputs; the observation of
// row r read from x + (xrow0 + r) * ldx (the global rows, or rows staged in LDS by the fused prologue).
// PRE: the wave's fragments already in registers (`pre`; the same MFMAs in the same order).
// the 16 values of a bias-table block that accumulator registers g = 4k + i of lane half h meet
// (feature mb * 32 + 8k + 4h + i, asvrl_mfma.h feat): four 16-byte LDS reads, issued together
__device__ __forceinline__ void bias16(const float* tab, int mb, int h, float (&b)[16]) {
  typedef float f4v __attribute__((ext_vector_type(4)));
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const f4v t = *reinterpret_cast<const f4v*>(tab + mb * 32 + 8 * k + 4 * h);
#pragma unroll
    for (int i = 0; i < 4; ++i) b[4 * k + i] = t[i];
  }
}

// object ob's mask factor (ob wave-uniform; -1, the self encoder, and kObjN give 1): selects on a scalar
// condition, no lane-divergent branches
static_assert(kSelfF >= 32 && kObjF >= 32, "a 32-feature block spans at most two encoders");
__device__ __forceinline__ float obj_sel(int ob, const float (&mf)[kObjN]) {
  float f = 1.f;
#pragma unroll
  for (int o = 0; o < kObjN; ++o) f = ob == o ? mf[o] : f;
  return f;
}

template <int MODE, bool PRE = false>
__device__ __forceinline__ void actor_split_tile(const MlpArgs& a, ActorSplitLds& L, int tile, const float* x,
                                                 int64_t ldx, int xrow0, const SplitPre& pre = SplitPre{}) {
  const AsvMlpIO& io = a.io;
  // w wave-uniform (an SGPR): the encoder epilogue's feature / object indices below are scalar work
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), h = lane >> 5,
            r = lane & 31;
  const int row = tile * 32 + r;
  const bool valid = row < io.n;
  const int rr = valid ? row : io.n - 1;
  // ---------------- encoders (wave w: blocks 2w, 2w + 1) -> h0
  {
    frag8 bx[2];
    float mk[kObjN];
    load_obs(x, ldx, xrow0 + (rr - tile * 32), h, bx, mk);
    PRO_STAMP(10);
    if (MODE == MLP_TRAIN && w == 0 && valid) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        *reinterpret_cast<frag8*>(bp(io.xb) + static_cast<int64_t>(row) * kObsK + ks * 16 + 8 * h) = bx[ks];
    }
    const frag8* ENC = reinterpret_cast<const frag8*>(a.w.enc_frag);
    const RowA<kEnc> RA(r, h);
    float mf[kObjN];   // masked_fill(mask < 0.5, 0) as a factor per object
#pragma unroll
    for (int o = 0; o < kObjN; ++o) mf[o] = mk[o] < 0.5f ? 0.f : 1.f;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int mb = 2 * w + q;
      float bb[16];
      bias16(L.bias + kSbEnc, mb, h, bb);
      // a 32-feature block spans at most two encoders: A (from its first feature) up to feature bnd, then
      // A + 1; the lane's feature 8k + i + 4h of the block is in A iff 8k + i < lim. One select per element.
      const int m_lo = mb * 32;
      const int obA = m_lo < kSelfF ? -1 : obj_of(m_lo);
      const int lim = kSelfF + kObjF * (obA + 1) - m_lo - 4 * h;
      const float fA = obj_sel(obA, mf), fB = obj_sel(obA + 1, mf);
      f32x16 acc = f32x16{};
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        acc = mfma(PRE ? pre.enc[2 * q + ks] : ENC[(mb * 2 + ks) * 64 + lane], bx[ks], acc);
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int g = 8 * s + j;
          v[j] = relu(acc[g] + bb[g]) * ((g & 3) + 8 * (g >> 2) < lim ? fA : fB);
        }
        rows(L.x0, RA, 0, 2 * mb + s, pack8(v));
        if constexpr (MODE == MLP_TRAIN)
          store16(valid ? bp(io.h0) + static_cast<int64_t>(row) * kEnc + mb * 32 + 16 * s : nullptr, v, h);
      }
      if (q == 0) PRO_STAMP(11);
    }
  }
  PRO_STAMP(5);
  __syncthreads();
  PRO_STAMP(6);
  // ---------------- hidden_layer (wave w: block w) -> h1
  {
    const frag8* W1 = reinterpret_cast<const frag8*>(a.w.w1_frag);
    const RowA<kEnc> RX(r, h);
    const RowA<kHid> RH(r, h);
    float bb[16];
    bias16(L.bias + kSbB1, w, h, bb);
    f32x16 acc = f32x16{};
    if constexpr (PRE) {
#pragma unroll
      for (int ks = 0; ks < kEnc / 16; ++ks) acc = mfma(pre.w1[ks], rowf(L.x0, RX, 0, ks), acc);
    } else {
      acc = wchain<kEnc / 16>(W1, w * 16, lane, L.x0, RX);
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = relu(acc[8 * s + j] + bb[8 * s + j]);
      rows(L.h1, RH, 0, 2 * w + s, pack8(v));
      if constexpr (MODE == MLP_TRAIN)
        store16(valid ? bp(io.h1) + static_cast<int64_t>(row) * kHid + w * 32 + 16 * s : nullptr, v, h);
    }
  }
  PRO_STAMP(7);
  __syncthreads();
  // ---------------- hidden_layer_2 (block w) -> h2, the output layer's partial sums over its features
  {
    const frag8* W2 = reinterpret_cast<const frag8*>(a.w.w2_frag);
    const RowA<kHid> RH(r, h);
    float bb[16], wo0[16], wo1[16];
    bias16(L.bias + kSbB2, w, h, bb);
    bias16(L.bias + kSbWout, w, h, wo0);
    bias16(L.bias + kSbWout + kHid, w, h, wo1);
    f32x16 acc = f32x16{};
    if constexpr (PRE) {
#pragma unroll
      for (int ks = 0; ks < kHid / 16; ++ks) acc = mfma(pre.w2[ks], rowf(L.h1, RH, 0, ks), acc);
    } else {
      acc = wchain<kHid / 16>(W2, w * 8, lane, L.h1, RH);
    }
    float p0 = 0.f, p1 = 0.f;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        v[j] = relu(acc[8 * s + j] + bb[8 * s + j]);
        p0 += wo0[8 * s + j] * v[j];
        p1 += wo1[8 * s + j] * v[j];
      }
      if constexpr (MODE == MLP_TRAIN)
        store16(valid ? bp(io.h2) + static_cast<int64_t>(row) * kHid + w * 32 + 16 * s : nullptr, v, h);
    }
    p0 = half_sum(p0);
    p1 = half_sum(p1);
    if (h == 0) {
      L.part[w][r][0] = p0;
      L.part[w][r][1] = p1;
    }
  }
  PRO_STAMP(8);
  __syncthreads();
  PRO_STAMP(9);
  if (threadIdx.x >= 32 || !valid) return;
  const float z0 = (((L.part[0][r][0] + L.part[1][r][0]) + L.part[2][r][0]) + L.part[3][r][0]) + L.bias[kSbBout];
  const float z1 = (((L.part[0][r][1] + L.part[1][r][1]) + L.part[2][r][1]) + L.part[3][r][1]) + L.bias[kSbBout + 1];
  const float a0 = a.w.out_scale * atanf(z0);   // atan_scale * torch.atan(actions)
  const float a1 = a.w.out_scale * atanf(z1);
  float* o = io.a_out + static_cast<int64_t>(row) * io.ld_aout;
  o[0] = a0;
  o[1] = a1;
  if (MODE == MLP_TRAIN) {
    io.pre[static_cast<int64_t>(row) * 2] = z0;
    io.pre[static_cast<int64_t>(row) * 2 + 1] = z1;
  }
}

template <int MODE>
__global__ __launch_bounds__(kMlpWaves * 64) void actor_split_kernel(MlpArgs a) {
  __shared__ __attribute__((aligned(16))) ActorSplitLds L;
  SplitPre pre;
  split_prefetch(a.w, threadIdx.x >> 6, threadIdx.x & 63, pre);
  float bv[4];
  split_bias_fetch(a.w, threadIdx.x, bv);
  split_bias_store(L, threadIdx.x, bv);
  __syncthreads();
  actor_split_tile<MODE, true>(a, L, blockIdx.x, a.io.x, a.io.ldx, blockIdx.x * 32, pre);
}

// ------------------------------------------------------------------ fused learn prologue (AC-IQN)
// asvrl_replay_sample (B rows + the update's taus) + the local Actor's TRAIN forward on s
// (agent.py:419-421) + the target Actor's FWD on s' (agent.py:397-398) in ONE launch of 2 * B / 32
// workgroups: workgroup t < T draws samples 32 t .. 32 t + 31 (the same Philox draws as
// replay_sample_kernel), writes their rows and taus, and runs the TRAIN tile on the observations it
// staged in LDS; workgroup T + t draws the same samples, stages their next observations and runs the
// target FWD tile into na. Results are bit-identical to the three launches.
struct PrologueArgs {
  const float* ring;
  int64_t cap;
  const int64_t* ring_state;
  uint64_t seed, counter;
  const uint64_t* counter_dev;
  int64_t guard;
  int B, tau_sets, tau_n;
  float* out;
  float* taus;
};

__global__ __launch_bounds__(kMlpWaves * 64) void learn_prologue_kernel(PrologueArgs p, MlpArgs train, MlpArgs tgt) {
  PRO_STAMP(0);
  __shared__ __attribute__((aligned(16))) ActorSplitLds L;
  __shared__ __attribute__((aligned(16))) float xs[32 * ASVRL_OBS_DIM];   // the tile's 32 observation rows
  const int T = p.B / 32;
  const bool second = static_cast<int>(blockIdx.x) >= T;
  const int tile = second ? blockIdx.x - T : blockIdx.x;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  // the wave's weight fragments first: their L2 latency runs under the draw below
  SplitPre pre;
  split_prefetch(second ? tgt.w : train.w, w, lane, pre);
  float bv[4];
  split_bias_fetch(second ? tgt.w : train.w, threadIdx.x, bv);
  const int64_t head = p.ring_state[0], size = p.ring_state[1];
  const uint64_t ctr = p.counter + (p.counter_dev != nullptr ? *p.counter_dev : 0ull);
  // wave w gathers samples 8w .. 8w + 7 of the tile: the whole row to `out` (first half), the observation
  // (s, or s' for the second half) into LDS. Lanes 0..7 draw the eight slots at once; every row piece
  // (one float4 per lane) is loaded before any store, so the eight HBM reads are in flight together.
  const int64_t my_slot = replay_draw_slot(head, size, p.cap, p.guard, tile * 32 + 8 * w + (lane & 7), p.seed, ctr);
  const int slot_lo = static_cast<int>(my_slot & 0xFFFFFFFFll), slot_hi = static_cast<int>(my_slot >> 32);
  PRO_STAMP(1);
  constexpr int kRowV = ASVRL_TR_DIM / 4, kObsV = ASVRL_OBS_DIM / 4;
  const int per = second ? kObsV : kRowV;   // float4 pieces per sample
  typedef float f4v __attribute__((ext_vector_type(4)));
  f4v v[3];
  int jj[3], cc[3];
#pragma unroll
  for (int u = 0; u < 3; ++u) {   // every lane loads (pieces past the eight rows re-read row 0's): no
    const int e = lane + 64 * u;  // predicated loads, so v stays in registers
    jj[u] = e / per;
    cc[u] = e - jj[u] * per;
    const int js = jj[u] < 8 ? jj[u] : 0;
    const int64_t slot = (static_cast<int64_t>(__shfl(slot_hi, js)) << 32) |
                         static_cast<uint32_t>(__shfl(slot_lo, js));
    v[u] = reinterpret_cast<const f4v*>(p.ring + slot * ASVRL_TR_DIM)[(second ? kObsV : 0) + (jj[u] < 8 ? cc[u] : 0)];
  }
  PRO_STAMP(2);
  if (!second && p.taus != nullptr) {
    // the eight samples' taus with every lane busy: item (sample j, Philox block k0 / 4) per lane, the
    // draws of replay_draw_taus (same counters, bit-identical)
    const int per_row = p.tau_sets * p.tau_n, nblk = (per_row + 3) / 4;
    for (int it = lane; it < 8 * nblk; it += kWave) {
      const int j = it / nblk, k0 = 4 * (it - j * nblk), b = tile * 32 + 8 * w + j;
      const U4 r = philox4x32_10(U4{static_cast<uint32_t>(b), static_cast<uint32_t>(k0) ^ 0x7A0000u,
                                    static_cast<uint32_t>(ctr >> 32), static_cast<uint32_t>(ctr)},
                                 static_cast<uint32_t>(p.seed) ^ 0x51EDu, static_cast<uint32_t>(p.seed >> 32));
      const uint32_t rw[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int k = k0 + q;
        if (k < per_row) {
          const int set = k / p.tau_n, t = k - set * p.tau_n;
          p.taus[(static_cast<size_t>(set) * p.B + b) * p.tau_n + t] = static_cast<float>(rw[q] >> 8) * (1.0f / 16777216.0f);
        }
      }
    }
  }
#pragma unroll
  for (int u = 0; u < 3; ++u) {
    if (jj[u] < 8) {
      const int lr = 8 * w + jj[u], b = tile * 32 + lr;
      if (!second) reinterpret_cast<f4v*>(p.out + static_cast<size_t>(b) * ASVRL_TR_DIM)[cc[u]] = v[u];
      if (cc[u] < kObsV) reinterpret_cast<f4v*>(xs + lr * ASVRL_OBS_DIM)[cc[u]] = v[u];
    }
  }
  split_bias_store(L, threadIdx.x, bv);
  __syncthreads();
  PRO_STAMP(3);
  if (!second) actor_split_tile<MLP_TRAIN, true>(train, L, tile, xs, ASVRL_OBS_DIM, 0, pre);
  else actor_split_tile<MLP_FWD, true>(tgt, L, tile, xs, ASVRL_OBS_DIM, 0, pre);
  PRO_STAMP(4);
}

// The backward in the same split: dz2 (block w) from dA, dz1 = W2^T dz2 (block w), dz0 = W1^T dz1
// (blocks 2w, 2w + 1); the ReLU masks from the saved h2 / h1 / h0 of the lane's own features.
__device__ __forceinline__ void load_block16(const elem_t* rowp, int mb, int h, float (&v)[16]) {
#pragma unroll
  for (int g = 0; g < 16; g += 4) {
    float t[4];
    load4(rowp + mb * 32 + (g & 3) + 8 * (g >> 2) + 4 * h, t);
#pragma unroll
    for (int i = 0; i < 4; ++i) v[g + i] = t[i];
  }
}

__global__ __launch_bounds__(kMlpWaves * 64) void actor_bwd_split_kernel(MlpArgs a) {
  __shared__ __attribute__((aligned(16))) ActorSplitLds L;
  const AsvMlpIO& io = a.io;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 5, r = lane & 31;
  const int row = blockIdx.x * 32 + r;
  const bool valid = row < io.n;
  const int64_t rr = valid ? row : io.n - 1;
  elem_t* const dz2i = L.x0;
  elem_t* const dz1i = L.h1;
  // every weight fragment and saved activation the wave reads, fetched up front (one L2 / HBM latency for
  // the kernel instead of one per phase; the same MFMAs in the same order)
  frag8 w2t[kHid / 16], w1t[2][kHid / 16];
  {
    const frag8* W2T = reinterpret_cast<const frag8*>(a.w.w2t_frag);
    const frag8* W1T = reinterpret_cast<const frag8*>(a.w.w1t_frag);
#pragma unroll
    for (int ks = 0; ks < kHid / 16; ++ks) w2t[ks] = W2T[(w * 8 + ks) * 64 + lane];
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int ks = 0; ks < kHid / 16; ++ks) w1t[q][ks] = W1T[((2 * w + q) * 8 + ks) * 64 + lane];
  }
  float hv2[16], hv1[16], hv0[2][16];
  load_block16(bp(io.h2) + rr * kHid, w, h, hv2);
  load_block16(bp(io.h1) + rr * kHid, w, h, hv1);
#pragma unroll
  for (int q = 0; q < 2; ++q) load_block16(bp(io.h0) + rr * kEnc, 2 * w + q, h, hv0[q]);
  const float z0 = io.pre[rr * 2], z1 = io.pre[rr * 2 + 1];
  const float d0 = io.dA[rr * 2] * a.w.out_scale / (1.f + z0 * z0);
  const float d1 = io.dA[rr * 2 + 1] * a.w.out_scale / (1.f + z1 * z1);
  if (w == 0 && h == 0 && valid) {
    io.dout[row * 2] = d0;
    io.dout[row * 2 + 1] = d1;
  }
  const RowA<kHid> RH(r, h);
  // ---------------- dz2 (block w)
  {
    const float (&hv)[16] = hv2;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      float dv[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int m = feat(w, 8 * s + j, h);
        dv[j] = hv[8 * s + j] > 0.f ? a.w.wout[m] * d0 + a.w.wout[kHid + m] * d1 : 0.f;
      }
      rows(dz2i, RH, 0, 2 * w + s, pack8(dv));
      store16(valid ? bp(io.dz2) + rr * kHid + w * 32 + 16 * s : nullptr, dv, h);
    }
  }
  __syncthreads();
  // ---------------- dz1 = (W2^T dz2) 1[h1 > 0] (block w)
  {
    const float (&hv)[16] = hv1;
    f32x16 acc = f32x16{};
#pragma unroll
    for (int ks = 0; ks < kHid / 16; ++ks) acc = mfma(w2t[ks], rowf(dz2i, RH, 0, ks), acc);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      float dv[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) dv[j] = hv[8 * s + j] > 0.f ? acc[8 * s + j] : 0.f;
      rows(dz1i, RH, 0, 2 * w + s, pack8(dv));
      store16(valid ? bp(io.dz1) + rr * kHid + w * 32 + 16 * s : nullptr, dv, h);
    }
  }
  __syncthreads();
  // ---------------- dz0 = (W1^T dz1) 1[h0 > 0] (blocks 2w, 2w + 1)
  {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int mb = 2 * w + q;
      const float (&hv)[16] = hv0[q];
      f32x16 acc = f32x16{};
#pragma unroll
      for (int ks = 0; ks < kHid / 16; ++ks) acc = mfma(w1t[q][ks], rowf(dz1i, RH, 0, ks), acc);
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        float dv[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) dv[j] = hv[8 * s + j] > 0.f ? acc[8 * s + j] : 0.f;
        store16(valid ? bp(io.dz0) + rr * kEnc + mb * 32 + 16 * s : nullptr, dv, h);
      }
    }
  }
}

// ------------------------------------------------------------------ packing
// enc image (256 x 32, input-fed) from self_encoder / object_encoder, b_enc, the action-encoder
// image (128 x 16, input-fed, columns 2..15 zero) and the chained W1, W2, W2^T, W1^T images.
constexpr int kPackEnc = kEnc * kObsK, kPackAe = kHid * 16, kPackW1 = kHid * kEnc, kPackW2 = kHid * kHid;

__device__ __forceinline__ float enc_weight(const AsvMlpSrc& s, int m, int k) {
  if (m < kSelfF) return k < kSelfIn ? s.self_w[m * kSelfIn + k] : 0.f;
  const int o = obj_of(m), j = (m - kSelfF) % kObjF, c = k - kSelfIn - kObjIn * o;
  return (c >= 0 && c < kObjIn) ? s.obj_w[j * kObjIn + c] : 0.f;
}

__global__ __launch_bounds__(256) void mlp_pack_kernel(AsvMlpSrc src, AsvMlpWeights w) {
  int o = blockIdx.x * 256 + threadIdx.x;
  int row, col;
  if (o < kPackEnc) {
    frag_rc(o, kObsK, false, row, col);
    const_cast<elem_t*>(static_cast<const elem_t*>(w.enc_frag))[o] = (elem_t)enc_weight(src, row, col);
    if (o < kEnc)
      const_cast<float*>(w.b_enc)[o] = o < kSelfF ? src.self_b[o] : src.obj_b[(o - kSelfF) % kObjF];
    return;
  }
  o -= kPackEnc;
  if (o < kPackAe) {
    if (w.ae_frag == nullptr) return;
    frag_rc(o, 16, false, row, col);
    const_cast<elem_t*>(static_cast<const elem_t*>(w.ae_frag))[o] =
        (elem_t)(col < kNa ? src.ae_w[row * kNa + col] : 0.f);
    return;
  }
  o -= kPackAe;
  if (src.w1 == nullptr) return;
  if (o < kPackW1) {
    frag_rc(o, kEnc, true, row, col);
    const_cast<elem_t*>(static_cast<const elem_t*>(w.w1_frag))[o] = (elem_t)src.w1[row * kEnc + col];
    return;
  }
  o -= kPackW1;
  if (o < kPackW2) {
    frag_rc(o, kHid, true, row, col);
    const_cast<elem_t*>(static_cast<const elem_t*>(w.w2_frag))[o] = (elem_t)src.w2[row * kHid + col];
    return;
  }
  o -= kPackW2;
  if (o < kPackW2) {
    frag_rc(o, kHid, true, row, col);
    const_cast<elem_t*>(static_cast<const elem_t*>(w.w2t_frag))[o] = (elem_t)src.w2[col * kHid + row];
    return;
  }
  o -= kPackW2;
  if (o < kPackW1) {  // W1^T (256 x 128)
    frag_rc(o, kHid, true, row, col);
    const_cast<elem_t*>(static_cast<const elem_t*>(w.w1t_frag))[o] = (elem_t)src.w1[col * kEnc + row];
  }
}

// Encoder weight gradient (256 x 32 image) folded back onto the two Linear layers:
// self_w[m][k] = dW[m][k]; obj_w[j][c] = sum_o dW[56 + 40o + j][7 + 5o + c]; likewise biases.
__global__ __launch_bounds__(256) void enc_fold_kernel(const float* __restrict__ dw, const float* __restrict__ db,
                                                        float* self_w, float* self_b, float* obj_w, float* obj_b,
                                                        int accumulate) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  auto put = [&](float* p, float v) { *p = accumulate ? *p + v : v; };
  if (t < kSelfF * kSelfIn) {
    const int m = t / kSelfIn, k = t % kSelfIn;
    put(self_w + t, dw[m * kObsK + k]);
  } else if (t < kSelfF * kSelfIn + kObjF * kObjIn) {
    const int u = t - kSelfF * kSelfIn, j = u / kObjIn, c = u % kObjIn;
    float s = 0.f;
    for (int o = 0; o < kObjN; ++o) s += dw[(kSelfF + kObjF * o + j) * kObsK + kSelfIn + kObjIn * o + c];
    put(obj_w + u, s);
  } else if (t < kSelfF * kSelfIn + kObjF * kObjIn + kSelfF) {
    const int m = t - kSelfF * kSelfIn - kObjF * kObjIn;
    put(self_b + m, db[m]);
  } else if (t < kSelfF * kSelfIn + kObjF * kObjIn + kSelfF + kObjF) {
    const int j = t - kSelfF * kSelfIn - kObjF * kObjIn - kSelfF;
    float s = 0.f;
    for (int o = 0; o < kObjN; ++o) s += db[kSelfF + kObjF * o + j];
    put(obj_b + j, s);
  }
}

// dW[m][k] = sum_r dz[r][m] x[r][k], db[m] = sum_r dz[r][m] for a small f32 input (K <= 4): the
// critic action_encoder (2 -> 128). Block b handles rows [kSwRows*b, +kSwRows); thread t owns
// feature t % M and every (256/M)-th row, four rows in flight; partials [blk][M*K+M].
__global__ __launch_bounds__(256) void small_wgrad_kernel(const float* __restrict__ dz, int64_t ldz,
                                                           const float* __restrict__ x, int64_t ldx, int R, int M,
                                                           int K, float* __restrict__ partial) {
  __shared__ float red[256][5];
  small_wgrad_body(dz, ldz, x, ldx, R, M, K, partial, blockIdx.x, red);
}

}  // namespace
}  // namespace asvrl

using namespace asvrl;

extern "C" int asvrl_mlp_pack(const AsvMlpSrc* src, const AsvMlpWeights* w, void* stream) {
  ASVRL_REQUIRE(src && w && src->self_w && src->self_b && src->obj_w && src->obj_b && w->enc_frag && w->b_enc,
                "asvrl_mlp_pack: null argument");
  ASVRL_REQUIRE(!src->w1 || (src->w2 && w->w1_frag && w->w2_frag && w->w2t_frag && w->w1t_frag),
                "asvrl_mlp_pack: actor weights need all four hidden-layer images");
  ASVRL_REQUIRE(!w->ae_frag || src->ae_w, "asvrl_mlp_pack: action-encoder image without weights");
  const int total = kPackEnc + kPackAe + (src->w1 ? 2 * kPackW1 + 2 * kPackW2 : 0);
  hipLaunchKernelGGL(mlp_pack_kernel, dim3((total + 255) / 256), dim3(256), 0, as_stream(stream), *src, *w);
  return check_launch("asvrl_mlp_pack");
}

extern "C" int asvrl_mlp_encode(const AsvMlpWeights* w, const AsvMlpIO* io, void* stream) {
  ASVRL_REQUIRE(w && io && io->x && io->F && w->enc_frag && w->b_enc, "asvrl_mlp_encode: null argument");
  ASVRL_REQUIRE(!io->G || (io->act && w->ae_frag && w->b_ae), "asvrl_mlp_encode: G needs actions and ae weights");
  ASVRL_REQUIRE(io->ldx % 4 == 0 && reinterpret_cast<uintptr_t>(io->x) % 16 == 0,
                "asvrl_mlp_encode: obs rows must be 16-byte aligned");
  if (io->n <= 0) return 0;
  MlpArgs a{*w, *io};
  const int tiles = (io->n + 31) / 32;
  hipLaunchKernelGGL(encode_kernel, dim3((tiles + kMlpWaves - 1) / kMlpWaves), dim3(kMlpWaves * 64), 0,
                     as_stream(stream), a);
  return check_launch("asvrl_mlp_encode");
}

extern "C" int asvrl_actor_forward(const AsvMlpWeights* w, const AsvMlpIO* io, int32_t mode, void* stream) {
  ASVRL_REQUIRE(w && io && io->x && w->enc_frag && w->w1_frag && w->w2_frag && w->b1 && w->b2 && w->wout && w->bout,
                "asvrl_actor_forward: null argument");
  ASVRL_REQUIRE(mode == MLP_ACT || mode == MLP_FWD || mode == MLP_TRAIN, "asvrl_actor_forward: bad mode");
  ASVRL_REQUIRE(mode != MLP_ACT || io->a_out64, "asvrl_actor_forward: ACT needs a_out64");
  ASVRL_REQUIRE(mode == MLP_ACT || io->a_out, "asvrl_actor_forward: needs a_out");
  ASVRL_REQUIRE(mode != MLP_TRAIN || (io->xb && io->h0 && io->h1 && io->h2 && io->pre),
                "asvrl_actor_forward: TRAIN needs xb, h0, h1, h2, pre");
  ASVRL_REQUIRE(io->ldx % 4 == 0 && reinterpret_cast<uintptr_t>(io->x) % 16 == 0,
                "asvrl_actor_forward: obs rows must be 16-byte aligned");
  if (io->n <= 0) return 0;
  MlpArgs a{*w, *io};
  const int tiles = (io->n + 31) / 32;
  hipStream_t st = as_stream(stream);
  const dim3 sgrid(tiles), block(kMlpWaves * 64);
  if (mode == MLP_FWD) {
    hipLaunchKernelGGL(actor_split_kernel<MLP_FWD>, sgrid, block, 0, st, a);
  } else if (mode == MLP_TRAIN) {
    hipLaunchKernelGGL(actor_split_kernel<MLP_TRAIN>, sgrid, block, 0, st, a);
  } else {   // the rollout's act over every robot: the LDS-staged one-wave-per-tile form
    hipLaunchKernelGGL(actor_kernel<MLP_ACT>, dim3((tiles + kMlpWaves - 1) / kMlpWaves), block, 0, st, a);
  }
  return check_launch("asvrl_actor_forward");
}

extern "C" int asvrl_learn_prologue(const AsvSampleArgs* s, const AsvMlpWeights* actor, const AsvMlpIO* train_io,
                                    const AsvMlpWeights* target_actor, float* na, void* stream) {
  ASVRL_REQUIRE(s && actor && train_io && target_actor && na && s->ring && s->ring_state && s->out,
                "asvrl_learn_prologue: null argument");
  ASVRL_REQUIRE(s->capacity > 0 && s->B > 0 && s->B % 32 == 0, "asvrl_learn_prologue: B must be a positive multiple of 32");
  ASVRL_REQUIRE(s->taus == nullptr || (s->tau_sets >= 1 && s->tau_n >= 1), "asvrl_learn_prologue: bad tau shape");
  ASVRL_REQUIRE(train_io->n == s->B && train_io->a_out && train_io->xb && train_io->h0 && train_io->h1 && train_io->h2 &&
                    train_io->pre, "asvrl_learn_prologue: the TRAIN outputs (n = B, a_out, xb, h0, h1, h2, pre)");
  for (const AsvMlpWeights* w : {actor, target_actor})
    ASVRL_REQUIRE(w->enc_frag && w->w1_frag && w->w2_frag && w->b1 && w->b2 && w->wout && w->bout,
                  "asvrl_learn_prologue: null actor weight");
  PrologueArgs p{s->ring, s->capacity, s->ring_state, s->seed, s->counter, s->counter_dev, s->guard,
                 s->B, s->tau_sets, s->tau_n, s->out, s->taus};
  MlpArgs tr{*actor, *train_io};
  AsvMlpIO fio{};
  fio.n = s->B;
  fio.a_out = na;
  fio.ld_aout = 2;
  MlpArgs tg{*target_actor, fio};
  hipLaunchKernelGGL(learn_prologue_kernel, dim3(2 * (s->B / 32)), dim3(kMlpWaves * 64), 0, as_stream(stream), p, tr,
                     tg);
  return check_launch("asvrl_learn_prologue");
}

extern "C" int asvrl_actor_backward(const AsvMlpWeights* w, const AsvMlpIO* io, void* stream) {
  ASVRL_REQUIRE(w && io && w->w2t_frag && w->w1t_frag && w->wout && io->dA && io->pre && io->h0 && io->h1 &&
                    io->h2 && io->dout && io->dz2 && io->dz1 && io->dz0,
                "asvrl_actor_backward: null argument");
  if (io->n <= 0) return 0;
  MlpArgs a{*w, *io};
  const int tiles = (io->n + 31) / 32;
  hipLaunchKernelGGL(actor_bwd_split_kernel, dim3(tiles), dim3(kMlpWaves * 64), 0, as_stream(stream), a);
  return check_launch("asvrl_actor_backward");
}

extern "C" int asvrl_encoder_fold(const float* dw, const float* db, float* self_w, float* self_b, float* obj_w,
                                  float* obj_b, int32_t accumulate, void* stream) {
  ASVRL_REQUIRE(dw && db && self_w && self_b && obj_w && obj_b, "asvrl_encoder_fold: null argument");
  const int n = kSelfF * kSelfIn + kObjF * kObjIn + kSelfF + kObjF;
  hipLaunchKernelGGL(enc_fold_kernel, dim3((n + 255) / 256), dim3(256), 0, as_stream(stream), dw, db, self_w,
                     self_b, obj_w, obj_b, accumulate);
  return check_launch("asvrl_encoder_fold");
}

extern "C" int asvrl_small_wgrad_partial(const float* dz, int64_t ldz, const float* x, int64_t ldx, int32_t R,
                                         int32_t M, int32_t K, float* partial, int64_t partial_floats,
                                         int32_t* groups_out, void* stream) {
  ASVRL_REQUIRE(dz && x && partial && groups_out, "asvrl_small_wgrad: null argument");
  ASVRL_REQUIRE(M >= 1 && M <= 256 && 256 % M == 0 && K >= 1 && K <= 4, "asvrl_small_wgrad: M | 256, K <= 4");
  *groups_out = 0;
  if (R <= 0) return 0;
  const int groups = (R + kSwRows - 1) / kSwRows;
  ASVRL_REQUIRE(partial_floats >= static_cast<int64_t>(groups) * (M * K + M), "asvrl_small_wgrad: workspace too small");
  hipLaunchKernelGGL(small_wgrad_kernel, dim3(groups), dim3(256), 0, as_stream(stream), dz, ldz, x, ldx, R, M, K,
                     partial);
  *groups_out = groups;
  return check_launch("asvrl_small_wgrad");
}

extern "C" int asvrl_small_wgrad(const float* dz, int64_t ldz, const float* x, int64_t ldx, int32_t R, int32_t M,
                                 int32_t K, float* dw, float* db, int32_t accumulate, float* work, int64_t work_floats,
                                 void* stream) {
  ASVRL_REQUIRE(dw != nullptr, "asvrl_small_wgrad: null dw");
  int32_t groups = 0;
  if (int rc = asvrl_small_wgrad_partial(dz, ldz, x, ldx, R, M, K, work, work_floats, &groups, stream)) return rc;
  if (groups == 0) return 0;
  return launch_partial_sum(work, groups, M * K, M, dw, db, accumulate, as_stream(stream));
}
