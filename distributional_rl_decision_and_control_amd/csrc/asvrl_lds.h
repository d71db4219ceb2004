// asvrl_lds.h -- activation images in LDS for the feature-split persistent kernels
// (asvrl_critic_fused.hip, asvrl_rainbow_net.hip): "chained position" order, XOR-swizzled rows,
// row reads (B operands of the next layer) and transposed reads (the K = rows operand of a weight
// gradient), and the bias-placement convention of the two builds.
#pragma once
#include "asvrl_mfma.h"

namespace asvrl {

// feature <-> chained position inside 16-aligned groups: swap bits 2 and 3 (an involution)
__host__ __device__ constexpr int swap23(int f) { return (f & ~12) | ((f & 4) << 1) | ((f & 8) >> 1); }

// The XOR swizzle of row r: 16-byte chunk c of the row is stored at chunk c ^ swz(r). Chosen so that all three
// access shapes of the images are free of LDS bank conflicts (checked by tools/lds_swizzle_check.py, which simulates
// the lane groups of MI355X_MICROARCH.md's LDS table on every access the kernels make):
//   row reads  (ds_read_b128, B operands: 16-lane groups, 64 banks) -- swz distinct over each group's 16 rows;
//   transposed reads (ds_read_b64_tr_b16, 32-lane groups, 64 banks) -- swz >> 2 distinct over 4 consecutive rows;
//   row stores (ds_write_b128, activation images: 8 consecutive lanes = 8 rows, 32 banks) -- swz & 7 distinct over
//     8 consecutive rows.
// Rounds 2-5 used ((r & 3) << 2) | ((r >> 2) & 3) (P >= 128; P = 64 likewise), which met the first two only: every
// 16-byte activation store was 2-way conflicted, SQ_LDS_BANK_CONFLICT 2.29 M cycles per fused critic launch
// (profiles/r06e_pmc_*); the low two bits now also take bit 1 (bit 0 at P = 64) of the row.
template <int P>
__device__ __forceinline__ int swz(int r) {
  static_assert(P == 64 || P == 128 || P == 256, "swizzled images are 64, 128 or 256 positions wide");
  if constexpr (P == 64) return (((r >> 1) & 1) << 2) | (((r >> 2) & 3) ^ ((r & 1) << 1));   // 128-byte rows
  else return ((r & 3) << 2) | (((r >> 2) & 3) ^ (r & 2));                                    // 256- / 512-byte rows
}

// element offset of (row r, position p) in an image of P positions per row; p % 4 == 0 for the
// 8-byte transposed reads, p % 8 == 0 for 16-byte accesses
template <int P>
__device__ __forceinline__ int img_off(int r, int p) {
#if ASVRL_OPERAND_F32
  return r * P + p;
#else
  return r * P + (((p >> 3) ^ swz<P>(r)) << 3) + (p & 7);
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

// Per-lane byte bases of the swizzled images, computed once per phase so that every access is one XOR
// plus an immediate offset (the swizzle arithmetic per access was most of the kernel's VALU).
// Row access (row 32 j + r, positions 16 ks + 8 h .. + 7): (chunk ^ x(row)) with chunk = 2 ks + h
// equals 2 (ks ^ (x >> 1)) + (h ^ (x & 1)) below 16 chunks, and x(32 j + r) = x(r).

// a precomputed base (asvrl_critic_fused.hip keeps each lane's bases in an LDS table)
struct RawBase {};

template <int P>
struct RowA {
  int base;
  __device__ __forceinline__ RowA(RawBase, int b) : base(b) {}
  __device__ __forceinline__ RowA(int r, int h) {
#if ASVRL_OPERAND_F32
    base = (r * P + 8 * h) * 4;
#else
    const int x = swz<P>(r);
    base = r * P * 2 + 32 * (x >> 1) + 16 * (h ^ (x & 1));
#endif
  }
  __device__ __forceinline__ int at(int j, int ks) const {
#if ASVRL_OPERAND_F32
    return base + (j * 32 * P + 16 * ks) * 4;
#else
    return (base ^ (32 * (ks & 7))) + 256 * (ks >> 3) + j * 32 * P * 2;
#endif
  }
};

template <int P>
__device__ __forceinline__ frag8 rowf(const elem_t* img, const RowA<P>& A, int j, int ks) {
  return *reinterpret_cast<const frag8*>(reinterpret_cast<const char*>(img) + A.at(j, ks));
}

template <int P>
__device__ __forceinline__ void rows(elem_t* img, const RowA<P>& A, int j, int ks, const frag8& v) {
  *reinterpret_cast<frag8*>(reinterpret_cast<char*>(img) + A.at(j, ks)) = v;
}

// Transposed access (rows 16 kk .. + 15 x columns 32 n .. + 31, see tr_frag): the lane's two 4-row
// reads start at rows ro and ro + 4 (ro = 8 (g >> 1) + q) and column chunk 4 n + cp; below 16 chunks
// (4 n + cp) ^ x = 4 (n ^ (x >> 2)) + (cp ^ (x & 3)).
template <int P>
struct TrA {
  int lo, hi;
  __device__ __forceinline__ TrA(RawBase, int l, int u) : lo(l), hi(u) {}
  __device__ __forceinline__ TrA(int lane) {
#if ASVRL_OPERAND_F32
    lo = (8 * (lane >> 5) * P + (lane & 31)) * 4;
    hi = 0;
#else
    const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
    const int cp = 2 * (g & 1) + (p >> 1), ro = 8 * (g >> 1) + q;
    const int x0 = swz<P>(ro), x1 = swz<P>(ro + 4);
    lo = ro * P * 2 + 64 * (x0 >> 2) + 16 * (cp ^ (x0 & 3)) + 8 * (p & 1);
    hi = (ro + 4) * P * 2 + 64 * (x1 >> 2) + 16 * (cp ^ (x1 & 3)) + 8 * (p & 1);
#endif
  }
};

template <int P>
__device__ __forceinline__ frag8 trf(const elem_t* img, const TrA<P>& A, int kk, int n) {
  const char* b = reinterpret_cast<const char*>(img);
#if ASVRL_OPERAND_F32
  b += A.lo + (16 * kk * P + 32 * n) * 4;
  frag8 v;
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = *reinterpret_cast<const float*>(b + j * P * 4);
  return v;
#else
  typedef short s16x4 __attribute__((ext_vector_type(4)));
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  const int off = 256 * (n >> 2) + kk * 16 * P * 2;
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(b + ((A.lo ^ (64 * (n & 3))) + off)));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(b + ((A.hi ^ (64 * (n & 3))) + off)));
  const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(frag8, v);
#endif
}

// accumulator block initialised with a bias in position order: register 8s + i of lane half h is
// position base + 16 s + 8 h + i
// 8 consecutive f32 (positions p0 .. p0 + 7) from LDS as two 16-byte reads
__device__ __forceinline__ void lds8(const float* src, float (&v)[8]) {
  const f32x4 lo = *reinterpret_cast<const f32x4*>(src), hi = *reinterpret_cast<const f32x4*>(src + 4);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[i] = lo[i];
    v[4 + i] = hi[i];
  }
}

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

// Bias placement. bf16 build: the bias is the accumulator's initial value (no epilogue add). f32
// build (the parity build): zero initial value and the bias added after the dot product, the order
// of torch's addmm on the reference's CPU BLAS -- a pre-activation within rounding of 0 then takes
// the reference's side of the ReLU.
constexpr bool kBiasFirst = !ASVRL_OPERAND_F32;

__device__ __forceinline__ f32x16 acc_init(const float* bpos, int base, int h) {
  if constexpr (kBiasFirst) return bias_init(bpos, base, h);
  return f32x16{};
}

}  // namespace asvrl
