// asvrl_mfma.h -- shared MFMA helpers of the learner kernels (gfx950, wave64).
//
// Convention (v_mfma_f32_32x32x16_bf16): features are the MFMA M dimension, rows (samples) the
// N dimension. A 32x32 accumulator block has its row-of-batch on the lane (lane & 31) and its
// features in the 16 registers: register g of lane half h (= lane >> 5) holds feature
// (g & 3) + 8 (g >> 2) + 4 h of the block. Registers 8s..8s+7, converted to bf16, are directly
// the B operand of a following layer's k-step s ("chained" k order 16s + 8(j>>2) + 4h + (j&3));
// the A operand (weights) is pre-packed into per-lane fragments in that same k order.
//
// Operand type. The library is built twice from the same sources: libasvrl.so with bf16 operands
// (the training path) and libasvrl_f32.so with ASVRL_OPERAND_F32=1, where every operand, weight
// image and saved activation is f32 and each 32x32x16 bf16 MFMA becomes eight
// v_mfma_f32_32x32x2_f32 over the same fragments (instruction j takes element j of both operands,
// k = lane half: the k order is permuted identically on both sides, so the product is the same sum).
// The f32 build is the parity build of the hand-written learner (reference fp32 arithmetic).
// Its weight images are twice as large, so they are read from global memory (L2) instead of LDS.
#pragma once

#include <hip/hip_runtime.h>

#ifndef ASVRL_OPERAND_F32
#define ASVRL_OPERAND_F32 0
#endif

namespace asvrl {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#if ASVRL_OPERAND_F32
typedef float elem_t;   // MFMA operand / saved-activation / weight-image element
typedef f32x8 frag8;    // one lane's 8 operand elements of a 32x32x16 k-step
typedef f32x4 elem4;
constexpr bool kWeightsInLds = false;
__device__ __forceinline__ f32x16 mfma(frag8 a, frag8 b, f32x16 c) {
#pragma unroll
  for (int j = 0; j < 8; ++j) c = __builtin_amdgcn_mfma_f32_32x32x2f32(a[j], b[j], c, 0, 0, 0);
  return c;
}
#else
typedef __bf16 elem_t;
typedef bf16x8 frag8;
typedef bf16x4 elem4;
constexpr bool kWeightsInLds = true;
__device__ __forceinline__ f32x16 mfma(frag8 a, frag8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
#endif
constexpr int kElemBytes = static_cast<int>(sizeof(elem_t));

__device__ __forceinline__ elem_t* bp(void* p) { return reinterpret_cast<elem_t*>(p); }
__device__ __forceinline__ const elem_t* bp(const void* p) { return reinterpret_cast<const elem_t*>(p); }

// the weight image a kernel reads: its LDS copy (bf16 build) or the global image (f32 build)
__device__ __forceinline__ const frag8* wimg(const frag8* lds, const void* glob) {
  return kWeightsInLds ? lds : reinterpret_cast<const frag8*>(glob);
}
// LDS slots of a weight image: full size in the bf16 build, one fragment (unused) in the f32 build
constexpr int lds_frags(int n) { return kWeightsInLds ? n : 1; }

// Copy N fragments (global -> LDS) with the workgroup's T threads, up to CH per thread per batch: a
// batch's loads all issue before its stores (a plain strided loop waits for each load before its store,
// one L2 round trip per fragment and thread: ~5 us of a weight-staging workgroup's start)
template <int T, int N, int CH = 16>
__device__ __forceinline__ void copy_frags(frag8* dst, const frag8* __restrict__ src, int tid) {
  constexpr int PER = (N + T - 1) / T;
#pragma unroll
  for (int c0 = 0; c0 < PER; c0 += CH) {
    frag8 v[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int i = (c0 + c) * T + tid;
      if (c0 + c < PER && i < N) v[c] = src[i];
    }
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int i = (c0 + c) * T + tid;
      if (c0 + c < PER && i < N) dst[i] = v[c];
    }
  }
}

// feature index held by accumulator register g of 32-feature block mb in lane half h
__device__ __forceinline__ int feat(int mb, int g, int h) { return mb * 32 + (g & 3) + 8 * (g >> 2) + 4 * h; }

// full-mask DPP read (bound_ctrl set: lets the compiler fuse it into the consuming v_add_f32_dpp)
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, true));
}

// Sum over aligned groups of NT lanes (NT | 32), all on DPP: xor-1 and xor-2 quad butterflies,
// row_half_mirror (8), row_mirror (16) leave every lane of a 16-lane row with the row sum; for 32,
// row_bcast:15 (rows 1 and 3 only) adds the previous row's sum. The full sum is guaranteed in the
// LAST lane of each group (r % NT == NT - 1); for NT <= 16 every lane of the group has it.
template <int NT>
__device__ __forceinline__ float seg_sum(float v) {
  if (NT >= 2) v += dpp<0xB1>(v);   // quad_perm [1,0,3,2]
  if (NT >= 4) v += dpp<0x4E>(v);   // quad_perm [2,3,0,1]
  if (NT >= 8) v += dpp<0x141>(v);  // row_half_mirror
  if (NT >= 16) v += dpp<0x140>(v); // row_mirror
  if (NT >= 32)                     // row_bcast:15 into rows 1, 3 (rows 0, 2 add 0)
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x142, 0xA, 0xF, false));
  return v;
}

// One halving step of xreduce over lane bit K, partner lane by DPP control CTRL (a mirror or
// quad permutation that flips bit K and only bits below it): the lane with bit K clear keeps the
// lower half of x[0 .. n) plus its partner's, the other the upper half.
template <int CTRL, int K, int N>
__device__ __forceinline__ void xreduce_step(float* x, int lane) {
  const bool up = (lane >> K) & 1;
#pragma unroll
  for (int i = 0; i < N / 2; ++i) {
    const float lo = x[i] + dpp<CTRL>(x[i]);
    const float hi = x[i + N / 2] + dpp<CTRL>(x[i + N / 2]);
    x[i] = up ? hi : lo;
  }
}

// Transpose-reduce: sums each of the V values x[] over the aligned NT-lane groups of each lane
// half (NT | 32, NT <= V) by recursive halving, about V instructions in all instead of
// V * log2(NT). Afterwards x[0 .. V/NT) of lane r (= lane & 31) holds the group sums of the
// original values (r % NT) * (V/NT) + i. The 16-lane step is one v_permlane16_swap per pair: it
// leaves the two partial sums in its two results in every lane, so no select is needed.
template <int V, int NT>
__device__ __forceinline__ void xreduce(float (&x)[V], int lane) {
  static_assert(NT >= 2 && NT <= 32 && (NT & (NT - 1)) == 0 && V % NT == 0, "xreduce: NT | 32, NT <= V");
  if constexpr (NT >= 32) {   // bit 4: rows 0 <-> 1 of 16 lanes (and 2 <-> 3)
#pragma unroll
    for (int i = 0; i < V / 2; ++i) {
      const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x[i]), __float_as_uint(x[i + V / 2]), false,
                                                      false);
      x[i] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
    }
  }
  constexpr int N3 = NT >= 32 ? V / 2 : V;
  if constexpr (NT >= 16) xreduce_step<0x140, 3, N3>(x, lane);                   // row_mirror
  constexpr int N2 = NT >= 16 ? N3 / 2 : N3;
  if constexpr (NT >= 8) xreduce_step<0x141, 2, N2>(x, lane);                    // row_half_mirror
  constexpr int N1 = NT >= 8 ? N2 / 2 : N2;
  if constexpr (NT >= 4) xreduce_step<0x4E, 1, N1>(x, lane);                     // quad_perm [2,3,0,1]
  constexpr int N0 = NT >= 4 ? N1 / 2 : N1;
  xreduce_step<0xB1, 0, N0>(x, lane);                                            // quad_perm [1,0,3,2]
}

// x(lane) + x(lane ^ 32) in every lane, in the same order in both halves: one v_permlane32_swap of
// x with itself leaves (lower half's x, upper half's x) in the two results of every lane
__device__ __forceinline__ float half_sum(float x) {
  const unsigned u = __float_as_uint(x);
  const auto r = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// x(lane) + x(lane ^ 16) in every lane, the even 16-lane row's value first in both rows: one
// v_permlane16_swap of x with itself leaves (even row's x, odd row's x) in its two results (VALU; a
// __shfl_xor is an LDS ds_bpermute round trip)
__device__ __forceinline__ float row_pair_sum(float x) {
  const unsigned u = __float_as_uint(x);
  const auto r = __builtin_amdgcn_permlane16_swap(u, u, false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// cos(tau * pi * k) (Critic.calc_cos, AC_IQN_model.py:423) on the hardware cosine: v_cos_f32 takes
// revolutions, cos(2 pi x) with x = k tau / 2 (< 32 for k < 64, tau < 1: inside its +-256 domain).
// The value is rounded to bf16 for the MFMA right after, far above v_cos_f32's error. The f32 build
// computes the reference's expression itself: cos(tau * pis[k]) with pis[k] = f32(np.pi * k)
// (AC_IQN_model.py:389,423; IQN_model.py) and an f32 product.
__device__ __forceinline__ float cos_pi_k_tau(float tau, int k) {
#if ASVRL_OPERAND_F32
  const float pis = static_cast<float>(3.141592653589793 * static_cast<double>(k));
  return cosf(tau * pis);
#else
  return __builtin_amdgcn_cosf(tau * (0.5f * static_cast<float>(k)));
#endif
}

// cos(tau pi k) for k = k0 + 8 h + j, j < 8 (k0 a compile-time multiple of 16, h = lane half): bf16 build,
// x = tau (k / 2) = fma(tau, k0 / 2 + j / 2, tau * 4h) -- 4h is 0 or 4, so tau * 4h is exact and the fma's
// one rounding is the product's: bit-identical to cos_pi_k_tau, one VALU instruction per argument
// instead of three (int -> float, * 0.5, * tau)
__device__ __forceinline__ void cos_pi_k_tau8(float tau, int k0, int h, float (&c)[8]) {
#if ASVRL_OPERAND_F32
#pragma unroll
  for (int j = 0; j < 8; ++j) c[j] = cos_pi_k_tau(tau, k0 + 8 * h + j);
#else
  const float th = h ? 4.f * tau : 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) c[j] = __builtin_amdgcn_cosf(__builtin_fmaf(tau, 0.5f * static_cast<float>(k0 + j), th));
#endif
}

// the same for k = k0 + j, j < 8, with k0 known only at run time: k / 2 = k0 / 2 + j / 2 exactly (one add
// per argument instead of a conversion and a multiply), then the product with tau as in cos_pi_k_tau
__device__ __forceinline__ void cos_pi_k_tau8r(float tau, int k0, float (&c)[8]) {
#if ASVRL_OPERAND_F32
#pragma unroll
  for (int j = 0; j < 8; ++j) c[j] = cos_pi_k_tau(tau, k0 + j);
#else
  const float hb = 0.5f * static_cast<float>(k0);
#pragma unroll
  for (int j = 0; j < 8; ++j) c[j] = __builtin_amdgcn_cosf(tau * (hb + 0.5f * static_cast<float>(j)));
#endif
}

__device__ __forceinline__ float relu(float x) { return fmaxf(x, 0.f); }

// ReLU of 8 operand-typed values. bf16: a signed 16-bit max against 0 per half-word (v_pk_max_i16, two
// values per instruction): a bf16's sign is its int16 sign, so negatives and -0 become +0 and the rest
// stay, i.e. relu(round(x)) == round(relu(x)) bit for bit.
__device__ __forceinline__ frag8 relu_packed(frag8 v) {
#if ASVRL_OPERAND_F32
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = fmaxf(v[j], 0.f);
  return v;
#else
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  const s16x8 u = __builtin_elementwise_max(__builtin_bit_cast(s16x8, v), s16x8{});
  return __builtin_bit_cast(frag8, u);
#endif
}

// Eight f32 values to one operand fragment, converted two at a time: elements (2p, 2p + 1) by one
// v_cvt_pk_bf16_f32 into dword p. Written per element, the compiler converted the values one by one (a
// cvt against 0 each) or paired them off by one (1, 2), (3, 4), ... and repaired the halves with
// v_perm / v_alignbit: 2.5-4.5 VALU instructions per value instead of 0.5. Same rounding either way.
__device__ __forceinline__ frag8 pack8(const float (&v)[8]) {
#if ASVRL_OPERAND_F32
  frag8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = v[j];
  return r;
#else
  typedef float f2 __attribute__((ext_vector_type(2)));
  typedef __bf16 b2 __attribute__((ext_vector_type(2)));
  typedef unsigned u4 __attribute__((ext_vector_type(4)));
  u4 u;
#pragma unroll
  for (int p = 0; p < 4; ++p) u[p] = __builtin_bit_cast(unsigned, __builtin_convertvector(f2{v[2 * p], v[2 * p + 1]}, b2));
  return __builtin_bit_cast(frag8, u);
#endif
}

// v where m > 0, else +0 (m: operand values, e.g. a ReLU image): a bf16 is > 0 iff its half-word is > 0
// as int16, so t = min(max(m, 0) as int16, 1) as unsigned is 1 there and 0 elsewhere (-0 included), and
// the half-words of v times t are the selection -- three packed 16-bit instructions per two values
// (v_pk_max_i16, v_pk_min_u16, v_pk_mul_lo_u16) instead of a compare and a select each. Inline asm: in
// C the compiler sees through the multiply by 0 / 1 and emits the compares and selects again.
__device__ __forceinline__ frag8 mask_pos(frag8 v, frag8 m) {
#if ASVRL_OPERAND_F32
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = m[j] > 0.f ? v[j] : 0.f;
  return v;
#else
  typedef unsigned u4 __attribute__((ext_vector_type(4)));
  const u4 vu = __builtin_bit_cast(u4, v), mu = __builtin_bit_cast(u4, m);
  u4 r;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    unsigned t;
    asm("v_pk_max_i16 %0, %2, 0\n\tv_pk_min_u16 %0, %0, %3\n\tv_pk_mul_lo_u16 %0, %1, %0"
        : "=&v"(t)
        : "v"(vu[p]), "v"(mu[p]), "s"(0x00010001u));
    r[p] = t;
  }
  return __builtin_bit_cast(frag8, r);
#endif
}

// x[i] * y[i] for 8 values, two per v_pk_mul_f32 (the same f32 products)
__device__ __forceinline__ void mul8(const float (&x)[8], const float (&y)[8], float (&o)[8]) {
  typedef float f2 __attribute__((ext_vector_type(2)));
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const f2 r = f2{x[2 * p], x[2 * p + 1]} * f2{y[2 * p], y[2 * p + 1]};
    o[2 * p] = r.x;
    o[2 * p + 1] = r.y;
  }
}

// f32 accumulator of one 32-feature block initialised with the block's bias (natural feature order:
// register g of lane half h holds feature feat(mb, g, h), i.e. 4 consecutive biases per 16-byte load)
__device__ __forceinline__ f32x16 bias_nat(const float* b, int mb, int h) {
  f32x16 acc;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float4 v = *reinterpret_cast<const float4*>(b + mb * 32 + 8 * q + 4 * h);
    acc[4 * q] = v.x;
    acc[4 * q + 1] = v.y;
    acc[4 * q + 2] = v.z;
    acc[4 * q + 3] = v.w;
  }
  return acc;
}

// store of 4 consecutive features
__device__ __forceinline__ void store4(elem_t* base, const float* v) {
  elem4 x;
  x[0] = (elem_t)v[0];
  x[1] = (elem_t)v[1];
  x[2] = (elem_t)v[2];
  x[3] = (elem_t)v[3];
  *reinterpret_cast<elem4*>(base) = x;
}

// Store the 16 features of one k-step group (features 16s .. 16s+15 of a 32-feature block) of this
// lane's row: lane half h holds v = {4h .. 4h+3, 8+4h .. 8+4h+3}. v_permlane32_swap (one per
// dword, VALU, no LDS round trip) trades the upper half's features 4..7 against the lower half's
// 8..11, so half 0 then holds features 0..7 and half 1 features 8..15, and each lane writes one
// 16-byte piece: every row gets a full 32-byte sector per instruction. `grp` points at feature
// 16s of the row (nullptr: exchange only). All 64 lanes must call it.
__device__ __forceinline__ void store16(elem_t* grp, const float* v, int h) {
#if ASVRL_OPERAND_F32
  // f32: each lane writes its two 4-feature pieces (16 B each) directly
  if (grp != nullptr) {
    *reinterpret_cast<f32x4*>(grp + 4 * h) = f32x4{v[0], v[1], v[2], v[3]};
    *reinterpret_cast<f32x4*>(grp + 8 + 4 * h) = f32x4{v[4], v[5], v[6], v[7]};
  }
#else
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  const float (&v8)[8] = *reinterpret_cast<const float (*)[8]>(v);
  const u32x4 pk = __builtin_bit_cast(u32x4, pack8(v8));   // features 0..3 in dwords 0, 1; 4..7 in 2, 3
  const auto r0 = __builtin_amdgcn_permlane32_swap(pk[0], pk[2], false, false);
  const auto r1 = __builtin_amdgcn_permlane32_swap(pk[1], pk[3], false, false);
  const u32x4 out = {r0[0], r1[0], r0[1], r1[1]};
  if (grp != nullptr) *reinterpret_cast<u32x4*>(grp + 8 * h) = out;
#endif
}

// 4 consecutive elements -> f32
__device__ __forceinline__ void load4(const elem_t* base, float* v) {
  const elem4 x = *reinterpret_cast<const elem4*>(base);
  v[0] = static_cast<float>(x[0]);
  v[1] = static_cast<float>(x[1]);
  v[2] = static_cast<float>(x[2]);
  v[3] = static_cast<float>(x[3]);
}

// Fragment image element o of an (M x K) weight: ((mb*KS + ks)*64 + lane)*8 + j holds
// W[mb*32 + (lane&31)][col] with col = ks*16 + 8h + j (input-fed layer) or
// ks*16 + 8(j>>2) + 4h + (j&3) (chained layer).
__device__ __forceinline__ void frag_rc(int o, int K, bool chained, int& row, int& col) {
  const int j = o & 7, lane = (o >> 3) & 63, blk = o >> 9;
  const int KS = K / 16;
  const int ks = blk % KS, mb = blk / KS, h = lane >> 5;
  row = mb * 32 + (lane & 31);
  col = ks * 16 + (chained ? (8 * (j >> 2) + 4 * h + (j & 3)) : (8 * h + j));
}

}  // namespace asvrl
