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
#include "asvrl_common.h"
#include "asvrl_mfma.h"

namespace asvrl {
namespace {

constexpr int kC = 256, kH = 128, kNcos = 64, kNW = 4;

#if ASVRL_OPERAND_F32
template <int NT> struct FusedNB { static constexpr int v = 1; };
#else
template <int NT> struct FusedNB { static constexpr int v = 2; };
#endif

// feature <-> chained position inside 16-aligned groups: swap bits 2 and 3 (an involution)
__host__ __device__ constexpr int swap23(int f) { return (f & ~12) | ((f & 4) << 1) | ((f & 8) >> 1); }

// element offset of (row r, position p) in an image of P positions per row; p % 4 == 0 for the
// 8-byte transposed reads, p % 8 == 0 for 16-byte accesses
template <int P>
__device__ __forceinline__ int img_off(int r, int p) {
#if ASVRL_OPERAND_F32
  return r * P + p;
#else
  const int ch = p >> 3;
  int x;
  if constexpr (P == 64) x = (((r >> 1) & 1) << 2) | ((r >> 2) & 3);    // 128-byte rows
  else x = ((r & 3) << 2) | ((r >> 2) & 3);                              // 256- / 512-byte rows
  return r * P + ((ch ^ x) << 3) + (p & 7);
#endif
}

// B operand of a forward layer: row r, positions p0 .. p0 + 7
template <int P>
__device__ __forceinline__ frag8 row_frag(const elem_t* img, int r, int p0) {
  return *reinterpret_cast<const frag8*>(img + img_off<P>(r, p0));
}

template <int P>
__device__ __forceinline__ void row_store(elem_t* img, int r, int p0, const frag8& v) {
  *reinterpret_cast<frag8*>(img + img_off<P>(r, p0)) = v;
}

// operand fragment "rows r0 .. r0+15 x columns c0 .. c0+31" read transposed: lane l gets column
// c0 + (l & 31), rows r0 + 8 (l >> 5) + j in element j (the K = rows operand of a weight gradient)
template <int P>
__device__ __forceinline__ frag8 tr_frag(const elem_t* img, int r0, int c0, int lane) {
#if ASVRL_OPERAND_F32
  const int col = c0 + (lane & 31), rb = r0 + 8 * (lane >> 5);
  frag8 v;
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = img[(rb + j) * P + col];
  return v;
#else
  typedef short s16x4 __attribute__((ext_vector_type(4)));
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int col = c0 + 16 * (g & 1) + 4 * p;
  const int row = r0 + 8 * (g >> 1) + q;
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + img_off<P>(row, col)));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + img_off<P>(row + 4, col)));
  const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(frag8, v);
#endif
}

// keep a fragment materialised in its packed operand form (4 VGPRs for bf16) while it lives across
// phases, instead of the compiler's choice of carrying the f32 values and rounding at the use
__device__ __forceinline__ void pin(frag8& v) {
  typedef unsigned int u32v __attribute__((ext_vector_type(sizeof(frag8) / 4)));
  u32v u = __builtin_bit_cast(u32v, v);
  asm volatile("" : "+v"(u));
  v = __builtin_bit_cast(frag8, u);
}

__device__ __forceinline__ float sum8(const frag8& v) {
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) s += static_cast<float>(v[j]);
  return s;
}

// accumulator block initialised with a bias in position order: register 8s + i of lane half h is
// position base + 16 s + 8 h + i
__device__ __forceinline__ f32x16 bias_init(const float* bpos, int base, int h) {
  f32x16 acc;
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const f32x4 lo = *reinterpret_cast<const f32x4*>(bpos + base + 16 * s + 8 * h);
    const f32x4 hi = *reinterpret_cast<const f32x4*>(bpos + base + 16 * s + 8 * h + 4);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      acc[8 * s + i] = lo[i];
      acc[8 * s + 4 + i] = hi[i];
    }
  }
  return acc;
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

// Bias placement. bf16 build: the bias is the accumulator's initial value (no epilogue add). f32
// build (the parity build): zero initial value and the bias added after the dot product, the order
// of torch's addmm on the reference's CPU BLAS -- a pre-activation within rounding of 0 then takes
// the reference's side of the ReLU.
constexpr bool kBiasFirst = !ASVRL_OPERAND_F32;

__device__ __forceinline__ f32x16 acc_init(const float* bpos, int base, int h) {
  if constexpr (kBiasFirst) return bias_init(bpos, base, h);
  return f32x16{};
}

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
};

template <int NB, int S>
struct FusedLds {
  elem_t cos[32 * NB * kNcos];   // natural order (the cos layer is input-fed)
  elem_t x[32 * NB * kC];        // F * c; after dW1: four waves' dzc images [G][64]
  elem_t a[32 * NB * kH];        // h1g, then dz1
  elem_t b[32 * NB * kH];        // dz2
  elem_t F[S * kC];              // position order
  float G[S * kH];               // position order
  float qpart[kNW][32 * NB];
  float dq[32 * NB];
  float bias[kC + 3 * kH];       // bc | b1 | b2 | wo, position order
  float red[kNW];
};

constexpr int kSelfF = 56, kSelfIn = 7, kObjF = 40, kObjIn = 5, kObsMask = 32;

// F (observation_processor, AC_IQN_model.py:284-308) and G (relu(action_encoder(a)),
// AC_IQN_model.py:468-470) of the round's S samples into LDS, position order; xb for the encoder
// weight gradient. f32 dot products in the same order as asvrl_critic.hip's stage_features.
template <int S>
__device__ __forceinline__ void stage_fg(const FusedArgs& a, int b0, elem_t* Fs, float* Gs) {
  for (int idx = threadIdx.x; idx < S * kC; idx += kNW * 64) {
    const int k = idx / kC, m = idx % kC;
    const float* x = a.obs + static_cast<int64_t>(b0 + k) * a.ld_obs;
    float v;
    if (m < kSelfF) {
      const float* w = a.w.self_w + m * kSelfIn;
      float d = 0.f;
#pragma unroll
      for (int i = 0; i < kSelfIn; ++i) d += w[i] * x[i];
      v = relu(d + a.w.self_b[m]);
    } else {
      const int o = (m - kSelfF) / kObjF, j = (m - kSelfF) % kObjF;
      const float* w = a.w.obj_w + j * kObjIn;
      const float* xo = x + kSelfIn + kObjIn * o;
      float d = 0.f;
#pragma unroll
      for (int i = 0; i < kObjIn; ++i) d += w[i] * xo[i];
      v = x[kObsMask + o] < 0.5f ? 0.f : relu(d + a.w.obj_b[j]);   // masked_fill(mask < 0.5, 0)
    }
    Fs[k * kC + swap23(m)] = (elem_t)v;
  }
  for (int idx = threadIdx.x; idx < S * kH; idx += kNW * 64) {
    const int k = idx / kH, m = idx % kH;
    const float a0 = a.ain[static_cast<int64_t>(b0 + k) * a.ld_ain], a1 = a.ain[static_cast<int64_t>(b0 + k) * a.ld_ain + 1];
    Gs[k * kH + swap23(m)] = relu((a.w.ae_w[2 * m] * a0 + a.w.ae_w[2 * m + 1] * a1) + a.w.ae_b[m]);
  }
  if (a.xb != nullptr)
    for (int idx = threadIdx.x; idx < S * 32; idx += kNW * 64) {
      const int k = idx / 32, c = idx % 32;
      bp(a.xb)[static_cast<int64_t>(b0 + k) * 32 + c] = (elem_t)a.obs[static_cast<int64_t>(b0 + k) * a.ld_obs + c];
    }
}

// quantile-Huber terms of one row against its sample's N' = NT targets r + gamma q_next (1 - d)
// (agent.py:399-412); lane half h takes half of them. Returns dq; *wl = the row's loss sum.
template <int NT>
__device__ __forceinline__ float row_loss_dq(const FusedArgs& a, int b, float tau, float q, int lane, float* wl_out) {
  const int r = lane & 31, h = lane >> 5;
  const float* qt = a.qn + static_cast<size_t>(b) * NT;
  const float rb = a.rew[b * a.ld_rd], nd = 1.0f - a.don[b * a.ld_rd];
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
  const float qv = qt[r % NT];
  const float own = rb + (a.gamma * qv) * nd;   // r + gamma * q_next * (1 - d)
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
  *wl_out = half_sum(wl) / kap;
  return -(half_sum(wg) / kap) * a.gscale;
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

template <int NT>
__global__ __launch_bounds__(kNW * 64) __attribute__((amdgpu_waves_per_eu(1, 1)))
void critic_fused_kernel(FusedArgs a) {
  constexpr int NB = FusedNB<NT>::v, G = 32 * NB, S = G / NT;
  __shared__ __attribute__((aligned(16))) FusedLds<NB, S> L;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 5, r = lane & 31;
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
    wop[swap23(i)] = a.w.wo[i];
  }

  // persistent per-wave weight-gradient accumulators (rows = this wave's features, positions)
  f32x16 dW2[4], dW1[8], dWc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) dW2[i] = dWc[i] = f32x16{};
#pragma unroll
  for (int i = 0; i < 8; ++i) dW1[i] = f32x16{};
  float db2 = 0.f, db1 = 0.f, dbc0 = 0.f, dbc1 = 0.f, dbo = 0.f;
  float dwo[16];
#pragma unroll
  for (int g = 0; g < 16; ++g) dwo[g] = 0.f;
  for (int t = blockIdx.x; t < a.rounds; t += gridDim.x) {
    // the lane indices re-derived through an opaque copy every round: otherwise every LDS / weight
    // address of the round body is loop-invariant, gets hoisted out of the loop and spills
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
    const int lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6), h = lane >> 5, r = lane & 31;
    elem_t* const dzc_w = L.x + w * G * kNcos;   // this wave's dzc image [G][64] (after dW1)
    const int row0 = t * G, b0 = row0 / NT;
    // ---------------- stage: F, G, xb; cos(tau pi k) for the round's rows (natural order)
    stage_fg<S>(a, b0, L.F, L.G);
    for (int c = threadIdx.x; c < G * (kNcos / 8); c += kNW * 64) {
      const int row = c / (kNcos / 8), ch = c % (kNcos / 8);
      const float tau = a.taus[row0 + row];
      frag8 v;
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (elem_t)cos_pi_k_tau(tau, 8 * ch + j);
      row_store<kNcos>(L.cos, row, 8 * ch, v);
    }
    __syncthreads();

    // ---------------- L0: c = relu(Wc cos + bc), x = F * c      (this wave: blocks 2w, 2w+1)
    {
    ASVRL_FRESH_LANE();
#pragma unroll
    for (int mq = 0; mq < 2; ++mq) {
      const int mb = 2 * w + mq;
      frag8 wa[4];
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) wa[ks] = WC[(mb * 4 + ks) * 64 + lane];
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        f32x16 acc = acc_init(bcp, mb * 32, h);
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) acc = mfma(wa[ks], row_frag<kNcos>(L.cos, 32 * j + r, 16 * ks + 8 * h), acc);
        if constexpr (!kBiasFirst) acc += bias_init(bcp, mb * 32, h);
        const int bl = (32 * j + r) / NT;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const int p0 = mb * 32 + 16 * s + 8 * h;
          const frag8 fv = *reinterpret_cast<const frag8*>(L.F + bl * kC + p0);
          frag8 xo;
#pragma unroll
          for (int i = 0; i < 8; ++i) xo[i] = (elem_t)(static_cast<float>(fv[i]) * relu(acc[8 * s + i]));
          row_store<kC>(L.x, 32 * j + r, p0, xo);
        }
      }
    }
    }
    __syncthreads();

    // ---------------- L1: h1 = relu(W1 x + b1) (own block w), h1g = h1 * G
    frag8 h1k[NB][2];
    {
      ASVRL_FRESH_LANE();
      f32x16 acc[NB];
#pragma unroll
      for (int j = 0; j < NB; ++j) acc[j] = acc_init(b1p, w * 32, h);
#pragma unroll
      for (int ks = 0; ks < kC / 16; ++ks) {
        const frag8 wa = W1[(w * 16 + ks) * 64 + lane];
#pragma unroll
        for (int j = 0; j < NB; ++j) acc[j] = mfma(wa, row_frag<kC>(L.x, 32 * j + r, 16 * ks + 8 * h), acc[j]);
      }
      if constexpr (!kBiasFirst)
#pragma unroll
        for (int j = 0; j < NB; ++j) acc[j] += bias_init(b1p, w * 32, h);
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        const int bl = (32 * j + r) / NT;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const int p0 = w * 32 + 16 * s + 8 * h;
          const f32x4 g0 = *reinterpret_cast<const f32x4*>(L.G + bl * kH + p0);
          const f32x4 g1 = *reinterpret_cast<const f32x4*>(L.G + bl * kH + p0 + 4);
          frag8 go;
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const float hv = relu(acc[j][8 * s + i]);
            h1k[j][s][i] = (elem_t)hv;
            go[i] = (elem_t)(hv * (i < 4 ? g0[i] : g1[i - 4]));
          }
          row_store<kH>(L.a, 32 * j + r, p0, go);
          pin(h1k[j][s]);
        }
      }
    }
    __syncthreads();

    // ---------------- L2: z2 = W2 h1g + b2 (own block w); partial q over its 32 features; h2 = relu(z2)
    // parked in the dz2 image (operand type) until dq is known
    {
      ASVRL_FRESH_LANE();
      f32x16 z2[NB];
#pragma unroll
      for (int j = 0; j < NB; ++j) z2[j] = acc_init(b2p, w * 32, h);
#pragma unroll
      for (int ks = 0; ks < kH / 16; ++ks) {
        const frag8 wa = W2[(w * 8 + ks) * 64 + lane];
#pragma unroll
        for (int j = 0; j < NB; ++j) z2[j] = mfma(wa, row_frag<kH>(L.a, 32 * j + r, 16 * ks + 8 * h), z2[j]);
      }
      if constexpr (!kBiasFirst)
#pragma unroll
        for (int j = 0; j < NB; ++j) z2[j] += bias_init(b2p, w * 32, h);
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        float part = 0.f;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const int p0 = w * 32 + 16 * s + 8 * h;
          frag8 hv;
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const float h2 = relu(z2[j][8 * s + i]);
            part += wop[p0 + i] * h2;
            hv[i] = (elem_t)h2;
          }
          row_store<kH>(L.b, 32 * j + r, p0, hv);
        }
        part = half_sum(part);
        if (h == 0) L.qpart[w][32 * j + r] = part;
      }
    }
    __syncthreads();

    // ---------------- loss: q = sum of the four partials + bo; quantile-Huber -> dq (row block j = w)
    {
    ASVRL_FRESH_LANE();
    for (int j = w; j < NB; j += kNW) {
      const int lr = 32 * j + r, grow = row0 + lr, b = grow / NT;
      const float q = (((L.qpart[0][lr] + L.qpart[1][lr]) + L.qpart[2][lr]) + L.qpart[3][lr]) + a.w.bo[0];
      float wl;
      const float dq = row_loss_dq<NT>(a, b, a.taus[grow], q, lane, &wl);
      if (a.tile_loss != nullptr) {
        float v = h == 0 ? wl : 0.f;
        v = seg_sum<32>(v);
        if (lane == 31) a.tile_loss[grow / 32] = v * a.loss_scale;
      }
      if (h == 0) {
        L.dq[lr] = dq;
        if (a.row_loss != nullptr) a.row_loss[grow] = wl;
        if (a.q != nullptr) a.q[grow] = q;
        dbo += dq;
      }
    }
    }
    __syncthreads();

    // ---------------- dz2 = dq wo 1[h2 > 0] (own block, in place over h2), output layer's gradient
    // sum of dq h2
    {
    ASVRL_FRESH_LANE();
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const float dqv = L.dq[32 * j + r];
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int p0 = w * 32 + 16 * s + 8 * h;
        const frag8 hv = row_frag<kH>(L.b, 32 * j + r, p0);
        frag8 dz;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const float h2 = static_cast<float>(hv[i]);
          dz[i] = (elem_t)(h2 > 0.f ? dqv * wop[p0 + i] : 0.f);
          dwo[8 * s + i] += dqv * h2;
        }
        row_store<kH>(L.b, 32 * j + r, p0, dz);
      }
    }
    }
    __syncthreads();

    // ---------------- dW2[own][:] += dz2^T h1g;  L3: dh1g = W2^T dz2 (own block)
    {
    ASVRL_FRESH_LANE();
#pragma unroll
    for (int kk = 0; kk < G / 16; ++kk) {
      const frag8 A = tr_frag<kH>(L.b, 16 * kk, 32 * w, lane);
      db2 += sum8(A);
#pragma unroll
      for (int n = 0; n < 4; ++n) mfma_acc(dW2[n], A, tr_frag<kH>(L.a, 16 * kk, 32 * n, lane));
    }
    }
    frag8 dz1k[NB][2];
    {
      ASVRL_FRESH_LANE();
      f32x16 acc[NB];
#pragma unroll
      for (int j = 0; j < NB; ++j) acc[j] = f32x16{};
#pragma unroll
      for (int ks = 0; ks < kH / 16; ++ks) {
        const frag8 wa = W2T[(w * 8 + ks) * 64 + lane];
#pragma unroll
        for (int j = 0; j < NB; ++j) acc[j] = mfma(wa, row_frag<kH>(L.b, 32 * j + r, 16 * ks + 8 * h), acc[j]);
      }
      // dz1 = dh1g G 1[h1 > 0]; dG = sum over the sample's taus of dh1g h1 (-> dzG = dG 1[G > 0])
#pragma unroll
      for (int j = 0; j < NB; ++j) {   // h1 unpacked here, not earlier
        pin(h1k[j][0]);
        pin(h1k[j][1]);
      }
      float gsa[NB][16];
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        const int bl = (32 * j + r) / NT;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const int p0 = w * 32 + 16 * s + 8 * h;
          const f32x4 g0 = *reinterpret_cast<const f32x4*>(L.G + bl * kH + p0);
          const f32x4 g1 = *reinterpret_cast<const f32x4*>(L.G + bl * kH + p0 + 4);
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const float h1 = static_cast<float>(h1k[j][s][i]);
            const float d = acc[j][8 * s + i];
            dz1k[j][s][i] = (elem_t)(h1 > 0.f ? d * (i < 4 ? g0[i] : g1[i - 4]) : 0.f);
            gsa[j][8 * s + i] = d * h1;
          }
        }
      }
      sample_sums<NT, NB>(gsa, w * 32, lane, [&](int bl, int p, float v) {
        const float gm = L.G[bl * kH + p];
        if (a.dzG != nullptr) a.dzG[static_cast<size_t>(b0 + bl) * kH + swap23(p)] = gm > 0.f ? v : 0.f;
      });
    }
    __syncthreads();   // every wave is past dW2 (h1g dead) and L3 (dz2 dead)
    {
      ASVRL_FRESH_LANE();
#pragma unroll
      for (int j = 0; j < NB; ++j)
#pragma unroll
        for (int s = 0; s < 2; ++s) row_store<kH>(L.a, 32 * j + r, w * 32 + 16 * s + 8 * h, dz1k[j][s]);
    }
    __syncthreads();

    // ---------------- dW1[own][:] += dz1^T x
    {
    ASVRL_FRESH_LANE();
#pragma unroll
    for (int kk = 0; kk < G / 16; ++kk) {
      const frag8 A = tr_frag<kH>(L.a, 16 * kk, 32 * w, lane);
      db1 += sum8(A);
#pragma unroll
      for (int n = 0; n < 8; ++n) mfma_acc(dW1[n], A, tr_frag<kC>(L.x, 16 * kk, 32 * n, lane));
    }
    }
    __syncthreads();   // x dead: the waves' dzc images take its place

    // ---------------- L4: dx = W1^T dz1 (own blocks 2w, 2w+1) with c = relu(Wc cos + bc) recomputed
    // (bit-identical to L0's); dF = sum over taus of dx c (-> dzF), dzc = dx F 1[c > 0]
    {
    ASVRL_FRESH_LANE();
#pragma unroll
    for (int mq = 0; mq < 2; ++mq) {
      const int mb = 2 * w + mq;
      frag8 wt[8], wc[4];
#pragma unroll
      for (int ks = 0; ks < 8; ++ks) wt[ks] = W1T[(mb * 8 + ks) * 64 + lane];
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) wc[ks] = WC[(mb * 4 + ks) * 64 + lane];
      float fsa[NB][16];
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        f32x16 dx = f32x16{};
#pragma unroll
        for (int ks = 0; ks < 8; ++ks) dx = mfma(wt[ks], row_frag<kH>(L.a, 32 * j + r, 16 * ks + 8 * h), dx);
        f32x16 cc = acc_init(bcp, mb * 32, h);
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) cc = mfma(wc[ks], row_frag<kNcos>(L.cos, 32 * j + r, 16 * ks + 8 * h), cc);
        if constexpr (!kBiasFirst) cc += bias_init(bcp, mb * 32, h);
        const int bl = (32 * j + r) / NT;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const int p0 = mb * 32 + 16 * s + 8 * h;
          const frag8 fv = *reinterpret_cast<const frag8*>(L.F + bl * kC + p0);
          frag8 dz;
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const float cv = static_cast<float>((elem_t)relu(cc[8 * s + i]));   // L0's bf16 c
            fsa[j][8 * s + i] = dx[8 * s + i] * cv;
            dz[i] = (elem_t)(cv > 0.f ? dx[8 * s + i] * static_cast<float>(fv[i]) : 0.f);
          }
          row_store<kNcos>(dzc_w, 32 * j + r, mq * 32 + 16 * s + 8 * h, dz);
        }
      }
      sample_sums<NT, NB>(fsa, mb * 32, lane, [&](int bl, int p, float v) {
        const float fm = static_cast<float>(L.F[bl * kC + p]);
        if (a.dzF != nullptr)
          bp(a.dzF)[static_cast<size_t>(b0 + bl) * kC + swap23(p)] = (elem_t)(fm > 0.f ? v : 0.f);
      });
    }

    }
    // ---------------- dWc[own 64][:] += dzc^T cos (this wave's own dzc image: in-order LDS, no barrier)
    {
    ASVRL_FRESH_LANE();
#pragma unroll
    for (int kk = 0; kk < G / 16; ++kk) {
      const frag8 A0 = tr_frag<kNcos>(dzc_w, 16 * kk, 0, lane);
      const frag8 A1 = tr_frag<kNcos>(dzc_w, 16 * kk, 32, lane);
      dbc0 += sum8(A0);
      dbc1 += sum8(A1);
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        const frag8 Bf = tr_frag<kNcos>(L.cos, 16 * kk, 32 * n, lane);
        mfma_acc(dWc[n], A0, Bf);
        mfma_acc(dWc[2 + n], A1, Bf);
      }
    }
    }
    __syncthreads();   // the next round overwrites cos, F, G, x
  }

  // ---------------- the workgroup's partials: [M*K + M] per layer, features in natural order
  mfma_drain();
  const int grp = blockIdx.x;
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
  db2 = half_sum(db2);
  db1 = half_sum(db1);
  dbc0 = half_sum(dbc0);
  dbc1 = half_sum(dbc1);
  if (h == 0) {
    p2[kH * kH + swap23(w * 32 + r)] = db2;
    p1[kH * kC + swap23(w * 32 + r)] = db1;
    pc[kC * kNcos + swap23(2 * w * 32 + r)] = dbc0;
    pc[kC * kNcos + swap23((2 * w + 1) * 32 + r)] = dbc1;
  }
  // output layer: sum over the half's 32 lanes (rows) of each register (feature), then the waves' dbo
  float* po = a.parts.out + static_cast<size_t>(grp) * (kH + 1);
#pragma unroll
  for (int g = 0; g < 16; ++g) {
    const float v = seg_sum<32>(dwo[g]);   // lane 31 of each half
    if (r == 31) po[swap23(w * 32 + 16 * (g >> 3) + 8 * h + (g & 7))] = v;
  }
  dbo = seg_sum<32>(h == 0 ? dbo : 0.f);
  if (lane == 31) L.red[w] = dbo;
  __syncthreads();
  if (threadIdx.x == 0) po[kH] = ((L.red[0] + L.red[1]) + L.red[2]) + L.red[3];
}

int cu_count() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
  }
  return n;
}

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

extern "C" int32_t asvrl_critic_fused_groups(int32_t B, int32_t N) {
  if (B <= 0 || (N != 8 && N != 16 && N != 32)) return 0;
  const int rounds = fused_rounds(B, N);
  return rounds < cu_count() ? rounds : cu_count();
}

extern "C" int asvrl_critic_train_fused(const AsvCriticWeights* w, const AsvCriticIO* io, const AsvCriticParts* parts,
                                        void* stream) {
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
  const int grid = asvrl_critic_fused_groups(io->B, io->N);
  hipStream_t st = as_stream(stream);
  if (io->N == 32) hipLaunchKernelGGL((critic_fused_kernel<32>), dim3(grid), dim3(kNW * 64), 0, st, a);
  else if (io->N == 16) hipLaunchKernelGGL((critic_fused_kernel<16>), dim3(grid), dim3(kNW * 64), 0, st, a);
  else hipLaunchKernelGGL((critic_fused_kernel<8>), dim3(grid), dim3(kNW * 64), 0, st, a);
  return check_launch("asvrl_critic_train_fused");
}
