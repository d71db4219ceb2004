// asvrl_wgrad.hip -- weight gradients of the learner's Linear layers on gfx950:
//   dW[m][k] = sum_r dZ[r][m] * X[r][k],   db[m] = sum_r dZ[r][m]
// over R rows of bf16 activations (the torch backward's grad_weight = dZ^T X and
// grad_bias = dZ.sum(0) of every nn.Linear on the path, AC_IQN_model.py:398-404, 476-479).
//
// The reduction runs over the ROW index, which is the memory-major index of both operands,
// so an MFMA operand fragment ("8 consecutive rows of one column") is a transposed read:
// each workgroup stages 32-row chunks of dZ and X into LDS with coalesced 16-byte loads
// (next chunk prefetched into registers while the current one is consumed) and feeds
// v_mfma_f32_32x32x16_bf16 from ds_read_b64_tr_b16. LDS rows are padded to a stride of
// 64 mod 256 bytes, which makes the 32-lane halves of every transposed read conflict-free.
// Each wave owns a fixed set of 32x32 output blocks for the whole R range of its workgroup;
// workgroups write f32 partials that a second launch sums in a fixed order (deterministic).
// The f32 build (ASVRL_OPERAND_F32, asvrl_mfma.h) stages f32 rows (4 per 16-byte chunk) and reads
// its operand fragments with plain LDS loads into the eight v_mfma_f32_32x32x2_f32 of mfma().
#include "asvrl_common.h"
#include "asvrl_mfma.h"

#include <algorithm>

namespace asvrl {
namespace {

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int kWgThreads = 256;
constexpr int kRC = 32;           // rows per staged chunk (2 MFMA k-steps)
constexpr int kMaxGroups = 256;
#ifndef ASVRL_WGRAD_PF
#define ASVRL_WGRAD_PF 1
#endif
constexpr int kPF = ASVRL_WGRAD_PF;   // staged chunks in flight per thread
static_assert(kPF >= 1 && kPF <= 4, "1..4 chunks in flight");
constexpr int kE16 = 16 / kElemBytes;   // elements per 16-byte staging chunk
typedef elem_t elem16B __attribute__((ext_vector_type(kE16)));

__host__ __device__ constexpr int lds_stride(int cols) {  // bytes, == 64 (mod 256)
  return ((kElemBytes * cols - 64 + 255) / 256) * 256 + 64;
}

// Operand fragment of rows [r0, r0 + 16) x columns [c0, c0 + 32) of a row-major LDS image:
// lane l gets column c0 + (l & 31), rows r0 + 8(l >> 5) + j, j = 0..7.
__device__ __forceinline__ frag8 frag_tr(const char* img, int stride, int r0, int c0, int lane) {
#if ASVRL_OPERAND_F32
  const int col = c0 + (lane & 31), rb = r0 + 8 * (lane >> 5);
  frag8 v;
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = *reinterpret_cast<const float*>(img + (rb + j) * stride + col * 4);
  return v;
#else
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int col = c0 + 16 * (g & 1) + 4 * p;
  const int row = r0 + 8 * (g >> 1) + q;
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  const char* a0 = img + row * stride + col * 2;
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0 + 4 * stride));
  const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(frag8, v);
#endif
}

template <int N, int STEP>
__device__ __forceinline__ void load_rows(u32x4 (&r)[N], const elem_t* __restrict__ base, int64_t ld, int64_t row,
                                          int c8) {
#pragma unroll
  for (int i = 0; i < N; ++i) r[i] = *reinterpret_cast<const u32x4*>(base + (row + i * STEP) * ld + c8 * kE16);
}

template <int M, int K, int W = 4>
struct Shape {
  static constexpr int T = W * 64;                          // threads per workgroup
  static constexpr int NMB = M / 32, NKB = K / 32, NB = NMB * NKB, NBW = NB / W;
  static constexpr bool kWide = NBW >= NKB;                // wave covers whole m-blocks
  static constexpr int NMW = kWide ? NBW / NKB : 1;        // m-blocks per wave
  static constexpr int NKW = kWide ? NKB : NBW;            // k-blocks per wave
  static constexpr int SZ = lds_stride(M), SX = lds_stride(K);
  static constexpr int NCZ = kRC * M / kE16, NCX = kRC * K / kE16;     // 16-B chunks per staged chunk
  static constexpr int CZ = NCZ >= T ? NCZ / T : 1;    // per thread (dZ)
  static constexpr int CX = NCX >= T ? NCX / T : 1;    // (X); fewer chunks than threads: some idle
  static_assert(M % 32 == 0 && K % 32 == 0 && NB % W == 0 && NBW >= 1, "block grid must split over the waves");
  static_assert(kWide ? (NBW % NKB == 0) : (NKB % NBW == 0), "wave blocks must tile rows or columns");
  static_assert(NCZ % T == 0 || T % NCZ == 0, "dZ chunks must tile the block");
  static_assert(NCX % T == 0 || T % NCX == 0, "X chunks must tile the block");
};

// One workgroup's share (`group`) of dW / db: chunks [group * per, (group + 1) * per) into its
// (M*K + M)-float partial. lz / lx / lbias: the workgroup's LDS (kRC*SZ, kRC*SX bytes, T x 8 floats).
template <int M, int K, int W>
__device__ __forceinline__ void wgrad_body(const elem_t* __restrict__ dz, int64_t ldz, const elem_t* __restrict__ x,
                                           int64_t ldx, int chunks, int chunks_per_group, float* __restrict__ partial,
                                           int group, char* lz, char* lx, float (*lbias)[8]) {
  using S = Shape<M, K, W>;
  constexpr int kT = S::T;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int c_beg = group * chunks_per_group;
  const int c_end = min(chunks, c_beg + chunks_per_group);

  // thread t always stages column chunk t % (M/kE16) (resp. K/kE16), rows t / (M/kE16) + i * (T*kE16/M)
  const int zc8 = t % (M / kE16), zr = t / (M / kE16);
  const int xc8 = t % (K / kE16), xr = t / (K / kE16);
  constexpr int ZRS = kT * kE16 / M, XRS = kT * kE16 / K;   // row step between a thread's chunks
  // threads past the shape's W waves (a 4-wave shape inside the 8-wave multi-layer launch) only
  // take part in the barriers
  const bool in_wg = t < kT;
  const bool zact = in_wg && t < S::NCZ, xact = in_wg && t < S::NCX;   // staging threads
  // PF chunks in flight per thread (registers), chunk c + PF loaded while chunk c is consumed;
  // the chunk order and the MFMA order are those of PF = 1 (bit-identical results)
  u32x4 rz[kPF][S::CZ], rx[kPF][S::CX];
  float bacc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  f32x16 acc[S::NMW * S::NKW];
#pragma unroll
  for (int i = 0; i < S::NMW * S::NKW; ++i) acc[i] = f32x16{};
  const int mb0 = S::kWide ? w * S::NMW : (w * S::NBW) / S::NKB;
  const int kb0 = S::kWide ? 0 : (w * S::NBW) % S::NKB;

  if (c_beg < c_end) {
#pragma unroll
    for (int b = 0; b < kPF; ++b) {   // chunk indices past the group's end reload its last chunk
      const int64_t cb = min(c_beg + b, c_end - 1);
      if (zact) load_rows<S::CZ, ZRS>(rz[b], dz, ldz, cb * kRC + zr, zc8);
      if (xact) load_rows<S::CX, XRS>(rx[b], x, ldx, cb * kRC + xr, xc8);
    }
  }
  for (int c0 = c_beg; c0 < c_end; c0 += kPF) {
#pragma unroll
    for (int b = 0; b < kPF; ++b) {
      const int c = c0 + b;
      if (c >= c_end) break;
      if (zact) {
#pragma unroll
        for (int i = 0; i < S::CZ; ++i) {
          *reinterpret_cast<u32x4*>(lz + (zr + i * ZRS) * S::SZ + zc8 * 16) = rz[b][i];
          const elem16B v = __builtin_bit_cast(elem16B, rz[b][i]);
#pragma unroll
          for (int j = 0; j < kE16; ++j) bacc[j] += static_cast<float>(v[j]);
        }
      }
      if (xact) {
#pragma unroll
        for (int i = 0; i < S::CX; ++i) *reinterpret_cast<u32x4*>(lx + (xr + i * XRS) * S::SX + xc8 * 16) = rx[b][i];
      }
      __syncthreads();
      if (c + kPF < c_end) {   // prefetch under the MFMAs
        if (zact) load_rows<S::CZ, ZRS>(rz[b], dz, ldz, static_cast<int64_t>(c + kPF) * kRC + zr, zc8);
        if (xact) load_rows<S::CX, XRS>(rx[b], x, ldx, static_cast<int64_t>(c + kPF) * kRC + xr, xc8);
      }
#pragma unroll
      for (int ks = 0; ks < kRC / 16; ++ks) {
        if (!in_wg) break;
        frag8 fa[S::NMW], fb[S::NKW];
#pragma unroll
        for (int i = 0; i < S::NMW; ++i) fa[i] = frag_tr(lz, S::SZ, ks * 16, (mb0 + i) * 32, lane);
#pragma unroll
        for (int j = 0; j < S::NKW; ++j) fb[j] = frag_tr(lx, S::SX, ks * 16, (kb0 + j) * 32, lane);
#pragma unroll
        for (int i = 0; i < S::NMW; ++i)
#pragma unroll
          for (int j = 0; j < S::NKW; ++j) acc[i * S::NKW + j] = mfma(fa[i], fb[j], acc[i * S::NKW + j]);
      }
      __syncthreads();
    }
  }

  // partial dW block (mb, kb): lane l holds column l&31, rows (reg&3) + 8(reg>>2) + 4h
  float* pw = partial + static_cast<int64_t>(group) * (M * K + M);
  const int h = lane >> 5, col = lane & 31;
  if (in_wg) {
#pragma unroll
    for (int i = 0; i < S::NMW; ++i)
#pragma unroll
      for (int j = 0; j < S::NKW; ++j)
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) {
          const int m = (mb0 + i) * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * h;
          pw[m * K + (kb0 + j) * 32 + col] = acc[i * S::NKW + j][reg];
        }
  }
  // partial db: threads sharing a column chunk fold their sums
#pragma unroll
  for (int j = 0; j < 8; ++j) lbias[t][j] = bacc[j];
  __syncthreads();
  if (t < M / kE16) {
    float s[kE16];
#pragma unroll
    for (int j = 0; j < kE16; ++j) s[j] = 0.f;
    for (int u = t; u < kT; u += M / kE16)
#pragma unroll
      for (int j = 0; j < kE16; ++j) s[j] += lbias[u][j];
#pragma unroll
    for (int j = 0; j < kE16; ++j) pw[M * K + t * kE16 + j] = s[j];
  }
}

template <int M, int K, int W>
__global__ __launch_bounds__(W * 64) void wgrad_kernel(const elem_t* __restrict__ dz, int64_t ldz,
                                                        const elem_t* __restrict__ x, int64_t ldx, int chunks,
                                                        int chunks_per_group, float* __restrict__ partial) {
  using S = Shape<M, K, W>;
  __shared__ __attribute__((aligned(16))) char lz[kRC * S::SZ];
  __shared__ __attribute__((aligned(16))) char lx[kRC * S::SX];
  __shared__ float lbias[S::T][8];
  wgrad_body<M, K, W>(dz, ldz, x, ldx, chunks, chunks_per_group, partial, blockIdx.x, lz, lx, lbias);
}

// dw[k] = sum_r dq[r] * X[r][k], db = sum_r dq[r] for an output layer with one unit.
// Thread t reads 16 bytes (8 columns) of row t / (K/8) + i * RP: RP rows in flight per block.
// Threads 0..255 work; every thread of the workgroup must call it. sa: 256 x 9 floats of LDS.
template <int K>
__device__ __forceinline__ void wgrad_vec_body(const float* __restrict__ dq, int64_t ldq, const elem_t* __restrict__ x,
                                               int64_t ldx, int R, int rows_per_group, float* __restrict__ partial,
                                               int group, float (*sa)[9]) {
  constexpr int C8 = K / 8, RP = kWgThreads / C8;
  const int t = threadIdx.x, c8 = t % C8, rr = t / C8;
  const int r_beg = group * rows_per_group, r_end = t < kWgThreads ? min(R, r_beg + rows_per_group) : 0;
  float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float b = 0.f;
  for (int r = r_beg + rr; r < r_end; r += RP) {
    const float d = dq[static_cast<int64_t>(r) * ldq];
    const frag8 v = *reinterpret_cast<const frag8*>(x + static_cast<int64_t>(r) * ldx + c8 * 8);
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] += d * static_cast<float>(v[j]);
    b += d;
  }
  if (t < kWgThreads) {
#pragma unroll
    for (int j = 0; j < 8; ++j) sa[t][j] = a[j];
    sa[t][8] = b;
  }
  __syncthreads();
  float* pw = partial + static_cast<int64_t>(group) * (K + 1);
  if (t < K) {   // column t = 8 * (t / 8) + t % 8 lives in threads with c8 == t / 8
    float s = 0.f;
    for (int u = t / 8; u < kWgThreads; u += C8) s += sa[u][t % 8];
    pw[t] = s;
  }
  if (t == 0) {
    float s = 0.f;
    for (int u = 0; u < kWgThreads; u += C8) s += sa[u][8];   // c8 == 0 threads saw every row once
    pw[K] = s;
  }
}

template <int K>
__global__ __launch_bounds__(kWgThreads) void wgrad_vec_kernel(const float* __restrict__ dq, int64_t ldq,
                                                                const elem_t* __restrict__ x, int64_t ldx, int R,
                                                                int rows_per_group, float* __restrict__ partial) {
  __shared__ float sa[kWgThreads][9];
  wgrad_vec_body<K>(dq, ldq, x, ldx, R, rows_per_group, partial, blockIdx.x, sa);
}

// Several layers in one launch (asvrl_linear_wgrad_multi): workgroup b belongs to the segment whose
// group range holds it and runs exactly the workgroup `b - first group` of that layer's own launch.
// Every shape here has 8 waves; the LDS is one buffer sized for the largest.
constexpr int kMultiW = 8;
enum WgShape { WG_256x64 = 0, WG_128x256, WG_128x128, WG_256x32, WG_32x128, WG_VEC128, WG_SMALL };
struct WgSeg {
  const void* dz;    // bf16 (MFMA shapes), f32 (WG_VEC128: dq with stride ldz; WG_SMALL)
  const void* x;     // bf16, f32 (WG_SMALL)
  int64_t ldz, ldx;
  float* partial;
  int chunks, per, shape, first;   // chunks / per: 32-row chunks (MFMA), rows (VEC), R (SMALL)
  int M, K;                        // WG_SMALL only
};
struct WgMulti {
  WgSeg s[ASVRL_MAX_WGRAD_SEGS];
  int n;
};
template <int M, int K, int W = kMultiW>
constexpr int stage_bytes() { return kRC * (Shape<M, K, W>::SZ + Shape<M, K, W>::SX); }
constexpr int cmax(int a, int b) { return a > b ? a : b; }
constexpr int kMultiStage = cmax(cmax(cmax(stage_bytes<256, 64>(), stage_bytes<128, 256>()),
                                      cmax(stage_bytes<128, 128>(), stage_bytes<256, 32>())),
                                 stage_bytes<32, 128, 4>());

template <int M, int K, int W = kMultiW>
__device__ __forceinline__ void multi_run(const WgSeg& g, int group, char* lds, float (*lbias)[8]) {
  using S = Shape<M, K, W>;
  wgrad_body<M, K, W>(static_cast<const elem_t*>(g.dz), g.ldz, static_cast<const elem_t*>(g.x), g.ldx,
                            g.chunks, g.per, g.partial, group, lds, lds + kRC * S::SZ, lbias);
}

#ifndef ASVRL_WGRAD_MULTI_WAVES
#define ASVRL_WGRAD_MULTI_WAVES 1
#endif
__global__ __launch_bounds__(kMultiW * 64, ASVRL_WGRAD_MULTI_WAVES) void wgrad_multi_kernel(WgMulti t) {
  __shared__ __attribute__((aligned(16))) char lds[kMultiStage];
  __shared__ float lbias[kMultiW * 64][8];
  const int b = blockIdx.x;
  int k = 0;
  while (k + 1 < t.n && b >= t.s[k + 1].first) ++k;
  const WgSeg& g = t.s[k];
  const int group = b - g.first;
  switch (g.shape) {
    case WG_256x64: multi_run<256, 64>(g, group, lds, lbias); break;
    case WG_128x256: multi_run<128, 256>(g, group, lds, lbias); break;
    case WG_128x128: multi_run<128, 128>(g, group, lds, lbias); break;
    case WG_256x32: multi_run<256, 32>(g, group, lds, lbias); break;
    case WG_32x128: multi_run<32, 128, 4>(g, group, lds, lbias); break;   // 4 of the 8 waves
    case WG_VEC128:
      wgrad_vec_body<128>(static_cast<const float*>(g.dz), g.ldz, static_cast<const elem_t*>(g.x), g.ldx, g.chunks,
                          g.per, g.partial, group, reinterpret_cast<float(*)[9]>(&lbias[0][0]));
      break;
    default:
      small_wgrad_body(static_cast<const float*>(g.dz), g.ldz, static_cast<const float*>(g.x), g.ldx, g.chunks, g.M,
                       g.K, g.partial, group, reinterpret_cast<float(*)[5]>(&lbias[0][0]));
      break;
  }
}

// Partial reductions: a block covers 64 outputs; its kSumWaves waves take groups
// k = kSumWaves u + wave with kSumAcc independent accumulators each, and the wave sums are folded
// by a fixed tree (deterministic, and the same order in every reduction launch).
#ifndef ASVRL_SUM_WAVES
#define ASVRL_SUM_WAVES 8
#endif
constexpr int kSumWaves = ASVRL_SUM_WAVES, kSumThreads = kSumWaves * 64;
static_assert(kSumWaves >= 2 && kSumWaves <= 16 && (kSumWaves & (kSumWaves - 1)) == 0, "power-of-two waves");

// pairwise tree over the wave sums: (((r0 + r1) + (r2 + r3)) + ...)
template <int W>
__device__ __forceinline__ float tree_at(float (*red)[64], int lane, int base) {
  if constexpr (W == 1) return red[base][lane];
  else return tree_at<W / 2>(red, lane, base) + tree_at<W / 2>(red, lane, base + W / 2);
}
__device__ __forceinline__ float sum_tree(float (*red)[64], int lane) { return tree_at<kSumWaves>(red, lane, 0); }

// A wave's share of the groups, k = wv + kSumWaves u, into kSumAcc accumulators (u mod kSumAcc:
// kSumAcc independent loads in flight per lane) folded by a fixed pairwise tree.
#ifndef ASVRL_SUM_ACC
#define ASVRL_SUM_ACC 8
#endif
constexpr int kSumAcc = ASVRL_SUM_ACC;
static_assert(kSumAcc >= 1 && (kSumAcc & (kSumAcc - 1)) == 0, "power-of-two accumulators");
template <int W>
__device__ __forceinline__ float acc_tree(const float* a, int base) {
  if constexpr (W == 1) return a[base];
  else return acc_tree<W / 2>(a, base) + acc_tree<W / 2>(a, base + W / 2);
}
__device__ __forceinline__ float wave_groups_sum(const float* __restrict__ p, int groups, int stride, int idx,
                                                 int wv) {
  float acc[kSumAcc];
#pragma unroll
  for (int a = 0; a < kSumAcc; ++a) acc[a] = 0.f;
  int k = wv;
  for (; k + (kSumAcc - 1) * kSumWaves < groups; k += kSumAcc * kSumWaves) {
#pragma unroll
    for (int a = 0; a < kSumAcc; ++a) acc[a] += p[static_cast<int64_t>(k + a * kSumWaves) * stride + idx];
  }
#pragma unroll
  for (int a = 0; a < kSumAcc; ++a)
    if (k + a * kSumWaves < groups) acc[a] += p[static_cast<int64_t>(k + a * kSumWaves) * stride + idx];
  return acc_tree<kSumAcc>(acc, 0);
}

// Fixed-order sum over the groups of partial[k * stride + idx] for this thread's lane. Every
// thread of the block must call it (it synchronises) and receives the same sum for its lane.
__device__ __forceinline__ float group_sum(const float* __restrict__ p, int groups, int stride, int idx, bool valid,
                                           int wv, int lane, float (*red)[64]) {
  red[wv][lane] = valid ? wave_groups_sum(p, groups, stride, idx, wv) : 0.f;
  __syncthreads();
  const float s = sum_tree(red, lane);
  __syncthreads();
  return s;
}

// out[i] (+)= sum_g partial[g][i], i < nw + nb (the trailing nb go to db).
__global__ __launch_bounds__(kSumThreads) void partial_sum_kernel(const float* __restrict__ partial, int groups,
                                                                   int nw, int nb, float* __restrict__ dw,
                                                                   float* __restrict__ db, int accumulate) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int i = blockIdx.x * 64 + lane;
  const int n = nw + nb;
  __shared__ float red[kSumWaves][64];
  const float s = group_sum(partial, groups, n, i, i < n, wv, lane, red);
  if (wv != 0 || i >= n) return;
  if (i >= nw && db == nullptr) return;
  float* o = i < nw ? dw + i : db + (i - nw);
  *o = accumulate ? *o + s : s;
}

// Several independent partial reductions in one launch: blockIdx.y = segment.
struct SumSegs {
  AsvPartialSum seg[ASVRL_MAX_SUM_SEGS];
  int slot0[ASVRL_MAX_SUM_SEGS];   // first norm slot of each segment's working blocks
  int nseg;
};

// group_sum for the five object copies of a fold output at once: one pass over the groups, each
// copy accumulated in group_sum's order (bit-identical to five group_sum calls), one tree
__device__ __forceinline__ void group_sum5(const float* __restrict__ p, int groups, int stride, const int* idx,
                                           const bool* valid, int wv, int lane, float (*red5)[kSumWaves][64],
                                           float* out) {
#pragma unroll
  for (int o = 0; o < 5; ++o) red5[o][wv][lane] = valid[o] ? wave_groups_sum(p, groups, stride, idx[o], wv) : 0.f;
  __syncthreads();
#pragma unroll
  for (int o = 0; o < 5; ++o) out[o] = sum_tree(red5[o], lane);
}

// ASVRL_SUM_FOLD_ENCODERS: output t of [self_w 56x7 | self_b 56 | obj_w 40x5 | obj_b 40] and the
// image entry of its o-th copy (self entries: o = 0 only), as asvrl_encoder_fold reads them
constexpr int kFoldSelfF = 56, kFoldSelfIn = 7, kFoldObjF = 40, kFoldObjIn = 5, kFoldObjN = 5, kFoldK = 32;
constexpr int kFoldOut = kFoldSelfF * kFoldSelfIn + kFoldSelfF + kFoldObjF * kFoldObjIn + kFoldObjF;
__device__ __forceinline__ bool fold_index(int t, int o, int boff, int& idx) {
  if (t < kFoldSelfF * kFoldSelfIn) {
    idx = (t / kFoldSelfIn) * kFoldK + t % kFoldSelfIn;
    return o == 0;
  }
  t -= kFoldSelfF * kFoldSelfIn;
  if (t < kFoldSelfF) {
    idx = boff + t;
    return o == 0;
  }
  t -= kFoldSelfF;
  if (t < kFoldObjF * kFoldObjIn) {
    const int j = t / kFoldObjIn, c = t % kFoldObjIn;
    idx = (kFoldSelfF + kFoldObjF * o + j) * kFoldK + kFoldSelfIn + kFoldObjIn * o + c;
    return true;
  }
  t -= kFoldObjF * kFoldObjIn;
  idx = boff + kFoldSelfF + kFoldObjF * o + t;
  return t < kFoldObjF;
}

// Outputs per lane of partial_sums_kernel: a block owns kSumSpan consecutive outputs, lane l the
// outputs base + 64 j + l. Every output is summed in group_sum's order. More than 1 measured slower
// (fewer waves in flight: 22.8 us at 1, 38.7 at 2, 51.4 at 4 for the critic's reduction).
#ifndef ASVRL_SUM_OPL
#define ASVRL_SUM_OPL 1
#endif
constexpr int kSumOpl = ASVRL_SUM_OPL, kSumSpan = 64 * kSumOpl;

__device__ __forceinline__ void group_sum_n(const float* __restrict__ p, int groups, int stride, const int* idx,
                                            const bool* valid, int wv, int lane, float (*red)[kSumWaves][64],
                                            float* out) {
#pragma unroll
  for (int j = 0; j < kSumOpl; ++j) red[j][wv][lane] = valid[j] ? wave_groups_sum(p, groups, stride, idx[j], wv) : 0.f;
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kSumOpl; ++j) out[j] = sum_tree(red[j], lane);
}

// Block x of a segment owns outputs [kSumSpan x, kSumSpan (x + 1)) (a scalar segment: block 0 alone,
// all threads). With sq_blocks, every block also writes the sum of the squares of the outputs it wrote
// (segments with norm = 1) to its slot (= its index), for asvrl_adam_step.
__global__ __launch_bounds__(kSumThreads) void partial_sums_kernel(SumSegs t, double* sq_blocks, float* step) {
  // one block per WORKING block of a segment (no empty blocks to dispatch): block b is block x of the
  // segment y whose working blocks [slot0[y], slot0[y + 1]) hold it
  int y = 0;
  while (y + 1 < t.nseg && static_cast<int>(blockIdx.x) >= t.slot0[y + 1]) ++y;
  const int bx = static_cast<int>(blockIdx.x) - t.slot0[y];
  const AsvPartialSum& g = t.seg[y];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  __shared__ float red[kSumOpl][kSumWaves][64];
  double sq = 0.0;
  const int n = g.nw + g.nb;
  if (n == 1) {   // scalar over many groups: the whole block, fixed order
    if (bx == 0) {
      float acc = 0.f;
      acc = strided_sum<float>(g.partial, threadIdx.x, g.groups, kSumThreads, acc);
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, kWave);
      if (lane == 0) red[0][wv][0] = acc;
      __syncthreads();
      if (threadIdx.x == 0) {
        const float s = sum_tree(red[0], 0);
        float* o = g.nw == 1 ? g.dw : g.db;
        *o = g.accumulate ? *o + s : s;
        if (g.norm) sq += static_cast<double>(*o) * *o;
      }
    }
  } else if (bx * kSumSpan < n) {   // block-uniform
    const int base = bx * kSumSpan + lane;
    const int stride = g.stride != 0 ? g.stride : n;
    const int boff = g.boff != 0 ? g.boff : g.nw;
    float s[kSumOpl];
    if (g.mode == ASVRL_SUM_FOLD_ENCODERS) {
      __shared__ float red5[kFoldObjN][kSumWaves][64];
      for (int j = 0; j < kSumOpl; ++j) {
        const int i = base + 64 * j;
        int idx[kFoldObjN];
        bool v[kFoldObjN];
        float so[kFoldObjN];
#pragma unroll
        for (int o = 0; o < kFoldObjN; ++o) {
          idx[o] = 0;
          v[o] = i < n && fold_index(i, o, boff, idx[o]);
        }
        group_sum5(g.partial, g.groups, stride, idx, v, wv, lane, red5, so);
        __syncthreads();   // red5 is rewritten by the next chunk
        s[j] = 0.f;   // the copies in object order (asvrl_encoder_fold)
#pragma unroll
        for (int o = 0; o < kFoldObjN; ++o)
          if (v[o]) s[j] += so[o];
      }
    } else {
      int idx[kSumOpl];
      bool v[kSumOpl];
#pragma unroll
      for (int j = 0; j < kSumOpl; ++j) {
        const int i = base + 64 * j;
        v[j] = i < n;
        idx[j] = i < g.nw ? i : boff + (i - g.nw);
      }
      group_sum_n(g.partial, g.groups, stride, idx, v, wv, lane, red, s);
    }
    if (wv == 0) {
#pragma unroll
      for (int j = 0; j < kSumOpl; ++j) {
        const int i = base + 64 * j;
        if (i < n && !(i >= g.nw && g.db == nullptr)) {
          float* o = i < g.nw ? g.dw + i : g.db + (i - g.nw);
          const float out = g.accumulate ? *o + s[j] : s[j];
          *o = out;
          if (g.norm) sq += static_cast<double>(out) * out;
        }
      }
    }
  }
  if (sq_blocks == nullptr) return;
  if (blockIdx.x == 0 && threadIdx.x == 0) step[0] += 1.f;   // read by the next launch
  // ---- squared norm: this working block's sum (wave 0 holds the outputs) into its own slot
  if (wv != 0) return;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) sq += __shfl_xor(sq, off, kWave);
  if (lane == 0) sq_blocks[blockIdx.x] = sq;
}

// norm slots: one per working block of each segment, segments in order
int norm_slots(const AsvPartialSum* segs, int nseg, int* slot0) {
  int n = 0;
  for (int k = 0; k < nseg; ++k) {
    if (slot0 != nullptr) slot0[k] = n;
    const int w = segs[k].nw + segs[k].nb;
    n += w == 1 ? 1 : (w + kSumSpan - 1) / kSumSpan;
  }
  return n;
}

int launch_partial_sums(const AsvPartialSum* segs, int nseg, double* sq_blocks, float* step, hipStream_t st) {
  SumSegs t{};
  for (int k = 0; k < nseg; ++k) {
    const AsvPartialSum& g = segs[k];
    ASVRL_REQUIRE(g.partial && g.dw && g.groups >= 0, "asvrl_partial_sums: null segment");
    ASVRL_REQUIRE(g.mode == ASVRL_SUM_PLAIN || g.mode == ASVRL_SUM_FOLD_ENCODERS, "asvrl_partial_sums: bad mode");
    ASVRL_REQUIRE(g.mode != ASVRL_SUM_FOLD_ENCODERS || (g.nw == kFoldOut && g.nb == 0),
                  "asvrl_partial_sums: the encoder fold writes 688 outputs (nw = 688, nb = 0)");
    t.seg[k] = g;
  }
  t.nseg = nseg;
  const int blocks = norm_slots(segs, nseg, t.slot0);
  hipLaunchKernelGGL(partial_sums_kernel, dim3(blocks), dim3(kSumThreads), 0, st, t, sq_blocks, step);
  return check_launch("asvrl_partial_sums");
}

// At least kMinChunks chunks per group: a small batch (the actor's B rows) would otherwise give a
// group per chunk and partials several times the size of the activations they reduce.
#ifndef ASVRL_WGRAD_MIN_CHUNKS
#define ASVRL_WGRAD_MIN_CHUNKS 4
#endif
constexpr int kMinChunks = ASVRL_WGRAD_MIN_CHUNKS;

// partial traffic is about groups * M * K floats: 2^ASVRL_WGRAD_CAP_LOG2 floats per layer at most
#ifndef ASVRL_WGRAD_CAP_LOG2
#define ASVRL_WGRAD_CAP_LOG2 23
#endif
int wgrad_groups(int R, int M, int K) {
  const int chunks = R / kRC;
  int cap = (1 << ASVRL_WGRAD_CAP_LOG2) / (M * K);
  cap = cap < 64 ? 64 : (cap > kMaxGroups ? kMaxGroups : cap);
  const int by_rows = (chunks + kMinChunks - 1) / kMinChunks;
  if (by_rows < cap) cap = by_rows;
  int groups = chunks < cap ? chunks : cap;
  if (groups < 1) return 0;
  const int per = (chunks + groups - 1) / groups;
  return (chunks + per - 1) / per;
}

int vec_groups(int R) {
  int groups = R < kMaxGroups ? R : kMaxGroups;
  if (groups < 1) return 0;
  const int per = (R + groups - 1) / groups;
  return (R + per - 1) / per;
}

template <int M, int K, int W = (M * K >= 8192 ? 8 : 4)>
int launch_wgrad(const elem_t* dz, int64_t ldz, const elem_t* x, int64_t ldx, int R, float* work, hipStream_t st,
                 int& groups) {
  // partial traffic is groups * M * K floats: capped near 32 MB for the large layers
  const int chunks = R / kRC;
  groups = wgrad_groups(R, M, K);
  const int per = (chunks + groups - 1) / groups;
  hipLaunchKernelGGL((wgrad_kernel<M, K, W>), dim3(groups), dim3(W * 64), 0, st, dz, ldz, x, ldx, chunks, per,
                     work);
  return check_launch("asvrl_linear_wgrad");
}

// ------------------------------------------------------------------ the Actor's gradients in ONE launch
// Every weight / bias gradient of the Actor (AC_IQN_model.py:284-321) from its backward's dZ and the
// TRAIN pass's saved activations over the B rows (agent.py:424-426: actor_loss.backward()), the actor
// loss, the squared-norm partials of clip_grad_norm_ and the Adam step count -- what wgrad_multi +
// partial_sums_norm did in two launches with per-group partials of the whole layer.
//
// Work items (one 4-wave workgroup each): a 32 x 32 output tile of hidden_layer_2 (16 tiles), hidden_layer
// (32) or the 256 x 32 encoder image (8), times S row splits of kAgRS rows; the output layer (S splits on
// the VALU); the loss. A tile item stages its split's dZ and X columns in LDS (each wave kAgRW rows, all
// loads issued at once), runs kAgRW / 16 MFMAs per wave (bias: one more MFMA against ones), folds the four
// waves in order and stores the split's 32 x 32 + 32 slab write-through (sc1). The LAST split of a tile to
// arrive (agent-scope counter, MI355X hand-off with sc1 stores / sc1 loads: no fence) sums the S slabs in
// split order -- the result does not depend on who arrives last -- writes the gradient and the tile's
// squared norm. The encoder image's eight tiles hand their merged tiles to the last of them, which folds
// the image onto self_encoder / object_encoder (sum over the five object copies in object order).
// Counters are left zero for the next launch (HIP-graph replay).
#if ASVRL_OPERAND_F32
constexpr int kAgRW = 32;    // rows per wave (f32 staging: 4x the bytes per row)
#else
constexpr int kAgRW = 128;
#endif
constexpr int kAgW = 4, kAgT = kAgW * 64, kAgRS = kAgW * kAgRW;   // waves, threads, rows per split
constexpr int kAgSt = lds_stride(32);                              // staged row stride (bytes)
constexpr int kAgCPR = 32 * kElemBytes / 16;                       // 16-byte chunks per staged row
constexpr int kAgNL = kAgRW * kAgCPR / 64;                         // chunks per lane per operand
static_assert(kAgNL >= 1 && (kAgRW * kAgCPR) % 64 == 0, "staging must tile the wave");
constexpr int kAgSlab = 32 * 32 + 32;                              // one split's tile + bias slab
constexpr int kAgT2 = 16, kAgT1 = 32, kAgTE = 8, kAgTiles = kAgT2 + kAgT1 + kAgTE;
constexpr int kAgOutItems = 16;   // output layer: one item per 8 of h2's 128 columns, over all rows
constexpr int kAgEncImg = 256 * 32 + 256;
constexpr int kAgCtrEnc = kAgTiles, kAgCounters = kAgTiles + 1;
constexpr int kAgSlotEnc = kAgT2 + kAgT1, kAgSlotOut = kAgSlotEnc + 1, kAgSlots = kAgSlotOut + kAgOutItems;
constexpr int kAgEncOut = 688;   // self_w 56x7 | self_b 56 | obj_w 40x5 | obj_b 40

// Phase timing (tools/ag_stamps.py; a variant build with -DASVRL_AG_STAMPS, never the shipped library):
// thread 0 of every workgroup records s_memrealtime (100 MHz, one clock for every CU) at its phase points.
#ifdef ASVRL_AG_STAMPS
constexpr int kAgStamps = 12;
__device__ uint64_t g_ag_stamps[4096 * kAgStamps];
#define AG_STAMP(k)                                                                          \
  do {                                                                                       \
    if (threadIdx.x == 0) g_ag_stamps[blockIdx.x * kAgStamps + (k)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define AG_STAMP(k) \
  do {              \
  } while (0)
#endif

struct AgLds {
  union {
    struct {
      char z[kAgW][kAgRW * kAgSt];
      char x[kAgW][kAgRW * kAgSt];
    } st;
    float cmb[kAgW][kAgSlab];
    float out[18][kAgT];      // output layer: [8 + 8 column sums, 2 bias sums][thread]
  } u;
  double red[kAgT];
  int last;
};

__device__ __forceinline__ float ld_sc1(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// every wave's slab stores have left, then one lane takes a ticket; true in the workgroup of the n-th
// arrival (the others return). The counter is reset by that workgroup.
__device__ __forceinline__ bool ag_arrive(int* cnt, int n, AgLds& L) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const int o = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    L.last = o == n - 1;
    if (o == n - 1) __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  return L.last != 0;
}

// fixed-order f64 sum of one value per thread; thread 0 gets the total
__device__ __forceinline__ double ag_block_sum(double v, AgLds& L) {
  L.red[threadIdx.x] = v;
  __syncthreads();
  for (int w = kAgT / 2; w > 0; w >>= 1) {
    if (static_cast<int>(threadIdx.x) < w) L.red[threadIdx.x] += L.red[threadIdx.x + w];
    __syncthreads();
  }
  return L.red[0];
}

// One tile item: dW[32 m][32 k] (+ db[32 m] when bias) over rows [r0, r0 + nch * kAgRS) of dz (columns
// m0..m0+31) and x (columns k0..k0+31), nch chunks of kAgRS rows. Returns true in the tile's last arriving
// workgroup, which then holds the S-split sum: thread t elements t + 256 j (m = e / 32, k = e % 32) in v[j],
// bias m = t in vb.
__device__ __forceinline__ bool ag_tile(const elem_t* __restrict__ dz, int ldz, const elem_t* __restrict__ x, int ldx,
                                        int R, int r0, int nch, bool bias, int S, int s, float* slabs, int* cnt,
                                        AgLds& L, float (&v)[4], float& vb) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  typedef unsigned int u32v4 __attribute__((ext_vector_type(4)));
  char* lz = L.u.st.z[w];
  char* lx = L.u.st.x[w];
  frag8 ones;
#pragma unroll
  for (int j = 0; j < 8; ++j) ones[j] = static_cast<elem_t>(1.0f);
  f32x16 acc = f32x16{}, accb = f32x16{};
  for (int ch = 0; ch < nch; ++ch) {
    const int rw0 = r0 + ch * kAgRS + w * kAgRW;
    u32v4 vz[kAgNL], vx[kAgNL];
#pragma unroll
    for (int i = 0; i < kAgNL; ++i) {   // all of the wave's loads in flight at once
      const int q = lane + 64 * i, row = q / kAgCPR, c = q % kAgCPR, gr = rw0 + row;
      const bool ok = gr < R;
      const int64_t g = ok ? gr : 0;
      vz[i] = *reinterpret_cast<const u32v4*>(dz + g * ldz + c * kE16);
      vx[i] = *reinterpret_cast<const u32v4*>(x + g * ldx + c * kE16);
      if (!ok) vz[i] = vx[i] = u32v4{0u, 0u, 0u, 0u};
    }
#pragma unroll
    for (int i = 0; i < kAgNL; ++i) {
      const int q = lane + 64 * i, row = q / kAgCPR, c = q % kAgCPR;
      *reinterpret_cast<u32v4*>(lz + row * kAgSt + c * 16) = vz[i];
      *reinterpret_cast<u32v4*>(lx + row * kAgSt + c * 16) = vx[i];
    }
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < kAgRW / 16; ++ks) {
      const frag8 A = frag_tr(lz, kAgSt, ks * 16, 0, lane);
      acc = mfma(A, frag_tr(lx, kAgSt, ks * 16, 0, lane), acc);
      if (bias) accb = mfma(A, ones, accb);
    }
    __syncthreads();   // the staging images are rewritten by the next chunk / reused as the fold area
  }
  AG_STAMP(1);
  const int h = lane >> 5, n = lane & 31;
  float* cw = L.u.cmb[w];
#pragma unroll
  for (int g = 0; g < 16; ++g) {
    const int m = (g & 3) + 8 * (g >> 2) + 4 * h;
    cw[m * 32 + n] = acc[g];
    if (bias && n == 0) cw[1024 + m] = accb[g];
  }
  __syncthreads();
  float* my = slabs + static_cast<size_t>(s) * kAgSlab;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int e = t + kAgT * j;
    v[j] = ((L.u.cmb[0][e] + L.u.cmb[1][e]) + L.u.cmb[2][e]) + L.u.cmb[3][e];
    if (S > 1) st_sc1(my + e, v[j]);
  }
  vb = 0.f;
  if (bias && t < 32) {
    vb = ((L.u.cmb[0][1024 + t] + L.u.cmb[1][1024 + t]) + L.u.cmb[2][1024 + t]) + L.u.cmb[3][1024 + t];
    if (S > 1) st_sc1(my + 1024 + t, vb);
  }
  if (S == 1) return true;
  AG_STAMP(2);
  if (!ag_arrive(cnt, S, L)) return false;
  AG_STAMP(3);
  // the S slabs in split order (this workgroup's own read back too), eight slabs' loads in flight at a time
  float acc4[4] = {0.f, 0.f, 0.f, 0.f}, accbs = 0.f;
  for (int s0 = 0; s0 < S; s0 += 8) {
    float u[8][4], ub[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const float* p = slabs + static_cast<size_t>(s0 + q < S ? s0 + q : s0) * kAgSlab;
#pragma unroll
      for (int j = 0; j < 4; ++j) u[q][j] = ld_sc1(p + t + kAgT * j);
      ub[q] = bias && t < 32 ? ld_sc1(p + 1024 + t) : 0.f;
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      if (s0 + q >= S) break;
#pragma unroll
      for (int j = 0; j < 4; ++j) acc4[j] = s0 + q == 0 ? u[q][j] : acc4[j] + u[q][j];
      accbs = s0 + q == 0 ? ub[q] : accbs + ub[q];
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) v[j] = acc4[j];
  vb = accbs;
  AG_STAMP(4);
  return true;
}

struct AgArgs {
  AsvActorGradIO io;
  int S, nch;   // row splits, kAgRS-row chunks per split
};

constexpr int kAgMaxEl = 5;   // outputs per thread of a finisher (tile: 4 + bias)

// A finisher's outputs (thread t: n of them, gradient addresses and values) are stored, and its squared
// norm goes to norm_parts[slot] (folded by the optimiser launch). (An optimiser step inside this launch, its
// finishers waiting for each other, was measured 22 us against 17 + 7 but could wait for minutes behind the
// kernels of other streams: profiles/r03p1_fused_adam_timeout.txt.)
__device__ __forceinline__ void ag_finish(const AgArgs& a, float* const (&dst)[kAgMaxEl], const float (&val)[kAgMaxEl],
                                          int n, int slot, AgLds& L) {
  const AsvActorGradIO& io = a.io;
  double sq = 0.0;
#pragma unroll
  for (int e = 0; e < kAgMaxEl; ++e) {
    if (e >= n) break;
    *dst[e] = val[e];
    sq += static_cast<double>(val[e]) * val[e];
  }
  sq = ag_block_sum(sq, L);
  if (threadIdx.x == 0 && io.norm_parts != nullptr) io.norm_parts[slot] = sq;
  AG_STAMP(5);
}

__global__ __launch_bounds__(kAgT) void actor_grads_kernel(AgArgs a) {
  __shared__ __attribute__((aligned(16))) AgLds L;
  const AsvActorGradIO& io = a.io;
  const int S = a.S, R = io.B, t = threadIdx.x;
  const int b = blockIdx.x;
  float* work = io.work;
  float* enc_img = work + static_cast<size_t>(kAgTiles) * S * kAgSlab;
#ifdef ASVRL_AG_STAMPS
  if (t == 0)
    for (int k = 1; k < kAgStamps; ++k) g_ag_stamps[blockIdx.x * kAgStamps + k] = 0;
#endif
  AG_STAMP(0);
  if (b == 0 && t == 0 && io.step != nullptr) io.step[0] += 1.f;   // read by the Adam launch
  float* dst[kAgMaxEl];
  float val[kAgMaxEl];
#pragma unroll
  for (int e = 0; e < kAgMaxEl; ++e) {
    dst[e] = nullptr;
    val[e] = 0.f;
  }
  if (b < kAgTiles * S) {
    const int tile = b / S, s = b % S;
    const elem_t *dz, *x;
    int ldz, ldx, mb, kb;
    if (tile < kAgT2) {   // hidden_layer_2: dz2 [R][128], h1 [R][128]
      dz = bp(io.dz2); ldz = 128; x = bp(io.h1); ldx = 128; mb = tile / 4; kb = tile % 4;
    } else if (tile < kAgT2 + kAgT1) {   // hidden_layer: dz1 [R][128], h0 [R][256]
      const int u = tile - kAgT2;
      dz = bp(io.dz1); ldz = 128; x = bp(io.h0); ldx = 256; mb = u / 8; kb = u % 8;
    } else {   // encoder image: dz0 [R][256], xb [R][32]
      dz = bp(io.dz0); ldz = 256; x = bp(io.xb); ldx = 32; mb = tile - kAgT2 - kAgT1; kb = 0;
    }
    const bool bias = kb == 0;
    float v[4], vb;
    if (!ag_tile(dz + mb * 32, ldz, x + kb * 32, ldx, R, s * a.nch * kAgRS, a.nch, bias, S, s,
                 work + static_cast<size_t>(tile) * S * kAgSlab, io.counters + tile, L, v, vb))
      return;
    if (tile < kAgT2 + kAgT1) {
      float* dw = tile < kAgT2 ? io.w2_grad : io.w1_grad;
      float* db = tile < kAgT2 ? io.b2_grad : io.b1_grad;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int e = t + kAgT * j, m = e >> 5, k = e & 31;
        dst[j] = dw + (mb * 32 + m) * ldx + kb * 32 + k;
        val[j] = v[j];
      }
      const int n = bias && t < 32 ? 5 : 4;
      dst[4] = db + mb * 32 + (t & 31);
      val[4] = vb;
      ag_finish(a, dst, val, n, tile, L);
      return;
    }
    // encoder image tile: to the shared image, then the last of the eight folds it
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int e = t + kAgT * j, m = e >> 5, k = e & 31;
      st_sc1(enc_img + (mb * 32 + m) * 32 + k, v[j]);
    }
    if (t < 32) st_sc1(enc_img + 256 * 32 + mb * 32 + t, vb);
    if (!ag_arrive(io.counters + kAgCtrEnc, kAgTE, L)) return;
    // thread t: outputs t, t + 256, t + 512 (< 688), each a sum of 1 or 5 image entries (object order);
    // every load issued before the sums
    constexpr int kEncPer = (kAgEncOut + kAgT - 1) / kAgT;
    float r5[kEncPer][5];
    int cnt5[kEncPer];
#pragma unroll
    for (int q = 0; q < kEncPer; ++q) {
      const int i = t + kAgT * q;
      int idx[5], c = 0;
      if (i < 56 * 7) {
        idx[0] = (i / 7) * 32 + i % 7; c = 1;
      } else if (i < 56 * 8) {
        idx[0] = 256 * 32 + (i - 56 * 7); c = 1;
      } else if (i < 56 * 8 + 40 * 5) {
        const int u = i - 56 * 8, j = u / 5, cc = u % 5;
#pragma unroll
        for (int o = 0; o < 5; ++o) idx[o] = (56 + 40 * o + j) * 32 + 7 + 5 * o + cc;
        c = 5;
      } else if (i < kAgEncOut) {
        const int j = i - 56 * 8 - 40 * 5;
#pragma unroll
        for (int o = 0; o < 5; ++o) idx[o] = 256 * 32 + 56 + 40 * o + j;
        c = 5;
      }
      cnt5[q] = c;
#pragma unroll
      for (int o = 0; o < 5; ++o) r5[q][o] = o < c ? ld_sc1(enc_img + idx[o]) : 0.f;
    }
    int n = 0;
#pragma unroll
    for (int q = 0; q < kEncPer; ++q) {
      if (cnt5[q] == 0) break;
      float r = r5[q][0];
#pragma unroll
      for (int o = 1; o < 5; ++o)
        if (o < cnt5[q]) r += r5[q][o];
      dst[q] = io.enc_grad + t + kAgT * q;
      val[q] = r;
      n = q + 1;
    }
    ag_finish(a, dst, val, n, kAgSlotEnc, L);
    return;
  }
  if (b < kAgTiles * S + kAgOutItems) {
    // output layer, columns 8j .. 8j + 7 of h2 over every row: dWo[a][k] = sum_r dout[r][a] h2[r][k] (and
    // item 0: dbo[a] = sum_r dout[r][a]); thread t takes rows t, t + 256, ... (eight in flight), then a fixed
    // pairwise tree over the threads -- no split, no slab
    const int j = b - kAgTiles * S, c0 = 8 * j;
    float a0[8], a1[8], b0 = 0.f, b1 = 0.f;
#pragma unroll
    for (int q = 0; q < 8; ++q) a0[q] = a1[q] = 0.f;
    const elem_t* h2 = bp(io.h2);
    constexpr int kRows = 16;   // rows in flight per thread (B = 4096: all of them, one memory round trip)
    for (int r = t; r < R; r += kAgT * kRows) {
      float2 d[kRows];
      frag8 hv[kRows];
#pragma unroll
      for (int u = 0; u < kRows; ++u) {
        const int ru = r + kAgT * u < R ? r + kAgT * u : r;
        d[u] = *reinterpret_cast<const float2*>(io.dout + 2 * static_cast<int64_t>(ru));
        hv[u] = *reinterpret_cast<const frag8*>(h2 + static_cast<int64_t>(ru) * 128 + c0);
      }
#pragma unroll
      for (int u = 0; u < kRows; ++u) {
        if (r + kAgT * u >= R) break;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const float hq = static_cast<float>(hv[u][q]);
          a0[q] += d[u].x * hq;
          a1[q] += d[u].y * hq;
        }
        b0 += d[u].x;
        b1 += d[u].y;
      }
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      L.u.out[q][t] = a0[q];
      L.u.out[8 + q][t] = a1[q];
    }
    L.u.out[16][t] = b0;
    L.u.out[17][t] = b1;
    AG_STAMP(1);
    __syncthreads();
    for (int w = kAgT / 2; w > 0; w >>= 1) {
      if (t < w)
#pragma unroll
        for (int q = 0; q < 18; ++q) L.u.out[q][t] += L.u.out[q][t + w];
      __syncthreads();
    }
    const int n = t < 16 || (j == 0 && t < 18) ? 1 : 0;   // weight row a = t / 8, column c0 + t % 8; bias a
    dst[0] = t < 16 ? io.wo_grad + (t >> 3) * 128 + c0 + (t & 7) : io.bo_grad + (t < 18 ? t - 16 : 0);
    val[0] = L.u.out[t < 18 ? t : 0][0];
    ag_finish(a, dst, val, n, kAgSlotOut + j, L);
    return;
  }
  // the actor loss: sum of the per-tile partials in a fixed order
  if (io.loss_out == nullptr || io.tile_loss == nullptr) return;
  float acc = 0.f;
  acc = strided_sum<float>(io.tile_loss, t, io.n_loss, kAgT, acc);
  const double tot = ag_block_sum(static_cast<double>(acc), L);
  if (t == 0) io.loss_out[0] = static_cast<float>(tot);
}

// Row splits (one chunk of kAgRS rows each at the bench shape); more rows per split only where the grid would
// pass 4096 workgroups (a very large B)
struct AgSplit {
  int S, nch;
};
AgSplit ag_split(int B) {
  const int chunks = (B + kAgRS - 1) / kAgRS;
  const int smax = (4096 - 1 - kAgOutItems) / kAgTiles;
  const int nch = (chunks + smax - 1) / smax;
  return AgSplit{(chunks + nch - 1) / nch, nch};
}

}  // namespace

int launch_partial_sum(const float* partial, int groups, int nw, int nb, float* dw, float* db, int accumulate,
                       hipStream_t st) {
  const int n = nw + nb;
  hipLaunchKernelGGL(partial_sum_kernel, dim3((n + 63) / 64), dim3(kSumThreads), 0, st, partial, groups, nw, nb, dw,
                     db, accumulate);
  return check_launch("partial_sum");
}

}  // namespace asvrl

using namespace asvrl;

extern "C" int32_t asvrl_linear_wgrad_groups(int32_t R, int32_t M, int32_t K) { return wgrad_groups(R, M, K); }
extern "C" int32_t asvrl_linear_wgrad_vec_groups(int32_t R) { return vec_groups(R); }

extern "C" int64_t asvrl_linear_wgrad_workspace(int32_t M, int32_t K) {
  return static_cast<int64_t>(kMaxGroups) * (static_cast<int64_t>(M) * K + M);
}

extern "C" int asvrl_linear_wgrad_partial(const void* dz, int64_t ldz, const void* x, int64_t ldx, int32_t R,
                                          int32_t M, int32_t K, float* partial, int64_t partial_floats,
                                          int32_t* groups_out, void* stream) {
  ASVRL_REQUIRE(dz && x && partial && groups_out, "asvrl_linear_wgrad: null argument");
  ASVRL_REQUIRE(R >= 0 && R % kRC == 0, "asvrl_linear_wgrad: R must be a multiple of 32");
  ASVRL_REQUIRE(ldz >= M && ldx >= K && ldz % 8 == 0 && ldx % 8 == 0,
                "asvrl_linear_wgrad: leading dimensions must cover the rows and be multiples of 8");
  ASVRL_REQUIRE((reinterpret_cast<uintptr_t>(dz) | reinterpret_cast<uintptr_t>(x)) % 16 == 0,
                "asvrl_linear_wgrad: operands must be 16-byte aligned");
  ASVRL_REQUIRE(partial_floats >= static_cast<int64_t>(wgrad_groups(R, M, K)) * (M * K + M),
                "asvrl_linear_wgrad: workspace too small");
  *groups_out = 0;
  if (R == 0) return 0;
  hipStream_t st = as_stream(stream);
  const elem_t* z = static_cast<const elem_t*>(dz);
  const elem_t* xx = static_cast<const elem_t*>(x);
  int groups = 0, rc = 0;
  if (M == 256 && K == 64) rc = launch_wgrad<256, 64>(z, ldz, xx, ldx, R, partial, st, groups);
  else if (M == 128 && K == 256) rc = launch_wgrad<128, 256>(z, ldz, xx, ldx, R, partial, st, groups);
  else if (M == 128 && K == 128) rc = launch_wgrad<128, 128>(z, ldz, xx, ldx, R, partial, st, groups);
  else if (M == 64 && K == 64) rc = launch_wgrad<64, 64>(z, ldz, xx, ldx, R, partial, st, groups);
  else if (M == 256 && K == 32) rc = launch_wgrad<256, 32>(z, ldz, xx, ldx, R, partial, st, groups);
  else if (M == 32 && K == 128) rc = launch_wgrad<32, 128>(z, ldz, xx, ldx, R, partial, st, groups);
  else ASVRL_REQUIRE(false, "asvrl_linear_wgrad: unsupported (M, K)");
  *groups_out = groups;
  return rc;
}

extern "C" int asvrl_linear_wgrad_multi(const AsvWgradSeg* segs, int32_t nseg, int32_t* groups_out, void* stream) {
  ASVRL_REQUIRE(segs && groups_out && nseg >= 0 && nseg <= ASVRL_MAX_WGRAD_SEGS,
                "asvrl_linear_wgrad_multi: bad segment table");
  WgMulti t{};
  int total = 0;
  for (int k = 0; k < nseg; ++k) {
    const AsvWgradSeg& a = segs[k];
    ASVRL_REQUIRE(a.dz && a.x && a.partial, "asvrl_linear_wgrad_multi: null argument");
    WgSeg& g = t.s[t.n];
    g.dz = a.dz; g.x = a.x; g.ldz = a.ldz; g.ldx = a.ldx; g.partial = a.partial; g.first = total;
    int groups = 0;
    if (a.kind != ASVRL_WGRAD_MFMA) {
      ASVRL_REQUIRE(a.R >= 0, "asvrl_linear_wgrad_multi: negative R");
      if (a.kind == ASVRL_WGRAD_VEC) {   // asvrl_linear_wgrad_vec_partial: dq f32 (stride ldz), x bf16, K = 128
        ASVRL_REQUIRE(a.M == 1 && a.K == 128 && a.ldx >= 128 && a.ldx % 8 == 0 &&
                          reinterpret_cast<uintptr_t>(a.x) % 16 == 0,
                      "asvrl_linear_wgrad_multi: vec segments need M = 1, K = 128, 16-byte aligned x");
        groups = a.R > 0 ? vec_groups(a.R) : 0;
        g.shape = WG_VEC128; g.chunks = a.R; g.per = groups ? (a.R + groups - 1) / groups : 1;
        ASVRL_REQUIRE(a.partial_floats >= static_cast<int64_t>(groups) * (a.K + 1),
                      "asvrl_linear_wgrad_multi: workspace too small");
      } else {   // asvrl_small_wgrad_partial: f32 dz (R x M) and x (R x K)
        ASVRL_REQUIRE(a.kind == ASVRL_WGRAD_SMALL, "asvrl_linear_wgrad_multi: bad kind");
        ASVRL_REQUIRE(a.M >= 1 && a.M <= 256 && 256 % a.M == 0 && a.K >= 1 && a.K <= 4,
                      "asvrl_linear_wgrad_multi: small segments need M | 256, K <= 4");
        groups = (a.R + kSwRows - 1) / kSwRows;
        g.shape = WG_SMALL; g.chunks = a.R; g.per = kSwRows; g.M = a.M; g.K = a.K;
        ASVRL_REQUIRE(a.partial_floats >= static_cast<int64_t>(groups) * (a.M * a.K + a.M),
                      "asvrl_linear_wgrad_multi: workspace too small");
      }
      groups_out[k] = groups;
      if (groups == 0) continue;
      ++t.n;
      total += groups;
      continue;
    }
    ASVRL_REQUIRE(a.R >= 0 && a.R % kRC == 0, "asvrl_linear_wgrad_multi: R must be a multiple of 32");
    ASVRL_REQUIRE(a.ldz >= a.M && a.ldx >= a.K && a.ldz % 8 == 0 && a.ldx % 8 == 0,
                  "asvrl_linear_wgrad_multi: leading dimensions must cover the rows and be multiples of 8");
    ASVRL_REQUIRE((reinterpret_cast<uintptr_t>(a.dz) | reinterpret_cast<uintptr_t>(a.x)) % 16 == 0,
                  "asvrl_linear_wgrad_multi: operands must be 16-byte aligned");
    int shape;
    if (a.M == 256 && a.K == 64) shape = WG_256x64;
    else if (a.M == 128 && a.K == 256) shape = WG_128x256;
    else if (a.M == 128 && a.K == 128) shape = WG_128x128;
    else if (a.M == 256 && a.K == 32) shape = WG_256x32;
    else if (a.M == 32 && a.K == 128) shape = WG_32x128;
    else ASVRL_REQUIRE(false,
                       "asvrl_linear_wgrad_multi: (M, K) must be (256,64), (128,256), (128,128), (256,32) or (32,128)");
    groups = a.R == 0 ? 0 : wgrad_groups(a.R, a.M, a.K);
    ASVRL_REQUIRE(a.partial_floats >= static_cast<int64_t>(groups) * (a.M * a.K + a.M),
                  "asvrl_linear_wgrad_multi: workspace too small");
    const int chunks = a.R / kRC;
    g.chunks = chunks; g.per = groups ? (chunks + groups - 1) / groups : 1; g.shape = shape;
    groups_out[k] = groups;
    if (groups == 0) continue;   // empty layers take no workgroups (and no table slot)
    ++t.n;
    total += groups;
  }
  if (total == 0) return 0;
  hipLaunchKernelGGL(wgrad_multi_kernel, dim3(total), dim3(kMultiW * 64), 0, as_stream(stream), t);
  return check_launch("asvrl_linear_wgrad_multi");
}

extern "C" int asvrl_linear_wgrad(const void* dz, int64_t ldz, const void* x, int64_t ldx, int32_t R, int32_t M,
                                  int32_t K, float* dw, float* db, int32_t accumulate, float* work,
                                  int64_t work_floats, void* stream) {
  ASVRL_REQUIRE(dw != nullptr, "asvrl_linear_wgrad: null dw");
  int32_t groups = 0;
  if (int rc = asvrl_linear_wgrad_partial(dz, ldz, x, ldx, R, M, K, work, work_floats, &groups, stream)) return rc;
  if (groups == 0) return 0;
  return launch_partial_sum(work, groups, M * K, M, dw, db, accumulate, as_stream(stream));
}

extern "C" int asvrl_partial_sums(const AsvPartialSum* segs, int32_t nseg, void* stream) {
  ASVRL_REQUIRE(segs && nseg >= 0 && nseg <= ASVRL_MAX_SUM_SEGS, "asvrl_partial_sums: bad segment table");
  if (nseg == 0) return 0;
  return launch_partial_sums(segs, nseg, nullptr, nullptr, as_stream(stream));
}

extern "C" int32_t asvrl_partial_sums_norm_parts(const AsvPartialSum* segs, int32_t nseg) {
  if (segs == nullptr || nseg <= 0 || nseg > ASVRL_MAX_SUM_SEGS) return 0;
  return norm_slots(segs, nseg, nullptr);
}

extern "C" int asvrl_partial_sums_norm(const AsvPartialSum* segs, int32_t nseg, double* norm_parts, float* step,
                                       void* stream) {
  ASVRL_REQUIRE(segs && nseg >= 1 && nseg <= ASVRL_MAX_SUM_SEGS, "asvrl_partial_sums_norm: bad segment table");
  ASVRL_REQUIRE(norm_parts && step, "asvrl_partial_sums_norm: null argument");
  return launch_partial_sums(segs, nseg, norm_parts, step, as_stream(stream));
}

extern "C" int asvrl_linear_wgrad_vec_partial(const float* dq, int64_t ldq, const void* x, int64_t ldx, int32_t R,
                                              int32_t K, float* partial, int64_t partial_floats, int32_t* groups_out,
                                              void* stream) {
  ASVRL_REQUIRE(dq && x && partial && groups_out, "asvrl_linear_wgrad_vec: null argument");
  ASVRL_REQUIRE(K == 128 || K == 256 || K == 64, "asvrl_linear_wgrad_vec: K must be 64, 128 or 256");
  ASVRL_REQUIRE(ldx >= K && ldx % 8 == 0 && reinterpret_cast<uintptr_t>(x) % 16 == 0,
                "asvrl_linear_wgrad_vec: x must be 16-byte aligned with ldx >= K, a multiple of 8");
  ASVRL_REQUIRE(partial_floats >= static_cast<int64_t>(vec_groups(R)) * (K + 1),
                "asvrl_linear_wgrad_vec: workspace too small");
  *groups_out = 0;
  if (R <= 0) return 0;
  hipStream_t st = as_stream(stream);
  const int groups = vec_groups(R);
  const int per = (R + groups - 1) / groups;
  const elem_t* xx = static_cast<const elem_t*>(x);
  if (K == 128) hipLaunchKernelGGL(wgrad_vec_kernel<128>, dim3(groups), dim3(kWgThreads), 0, st, dq, ldq, xx, ldx, R, per, partial);
  else if (K == 256) hipLaunchKernelGGL(wgrad_vec_kernel<256>, dim3(groups), dim3(kWgThreads), 0, st, dq, ldq, xx, ldx, R, per, partial);
  else hipLaunchKernelGGL(wgrad_vec_kernel<64>, dim3(groups), dim3(kWgThreads), 0, st, dq, ldq, xx, ldx, R, per, partial);
  *groups_out = groups;
  return check_launch("asvrl_linear_wgrad_vec");
}

extern "C" int asvrl_linear_wgrad_vec(const float* dq, int64_t ldq, const void* x, int64_t ldx, int32_t R, int32_t K,
                                      float* dw, float* db, int32_t accumulate, float* work, int64_t work_floats,
                                      void* stream) {
  ASVRL_REQUIRE(dw != nullptr, "asvrl_linear_wgrad_vec: null dw");
  int32_t groups = 0;
  if (int rc = asvrl_linear_wgrad_vec_partial(dq, ldq, x, ldx, R, K, work, work_floats, &groups, stream)) return rc;
  if (groups == 0) return 0;
  return launch_partial_sum(work, groups, K, 1, dw, db, accumulate, as_stream(stream));
}

#ifdef ASVRL_AG_STAMPS
extern "C" int asvrl_debug_ag_stamps(uint64_t* out, int64_t n) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ag_stamps), n * sizeof(uint64_t)) == hipSuccess ? 0 : 1;
}
extern "C" int asvrl_debug_ag_split(int32_t B, int32_t* out2) {
  const AgSplit sp = ag_split(B);
  out2[0] = sp.S;
  out2[1] = sp.nch;
  return 0;
}
#endif

extern "C" int64_t asvrl_actor_grads_workspace(int32_t B) {
  if (B <= 0) return 0;
  const int64_t S = ag_split(B).S;
  return static_cast<int64_t>(kAgTiles) * S * kAgSlab + kAgEncImg;
}
extern "C" int32_t asvrl_actor_grads_counters(void) { return kAgCounters; }
extern "C" int32_t asvrl_actor_grads_norm_parts(void) { return kAgSlots; }

namespace {
int check_actor_grads(const AsvActorGradIO* io) {
  ASVRL_REQUIRE(io && io->xb && io->h0 && io->h1 && io->h2 && io->dout && io->dz2 && io->dz1 && io->dz0,
                "asvrl_actor_grads: null activation");
  ASVRL_REQUIRE(io->w1_grad && io->b1_grad && io->w2_grad && io->b2_grad && io->wo_grad && io->bo_grad && io->enc_grad,
                "asvrl_actor_grads: null gradient");
  ASVRL_REQUIRE(io->work && io->counters, "asvrl_actor_grads: null workspace");
  ASVRL_REQUIRE(io->B >= 0 && io->n_loss >= 0, "asvrl_actor_grads: negative size");
  ASVRL_REQUIRE(io->work_floats >= asvrl_actor_grads_workspace(io->B), "asvrl_actor_grads: workspace too small");
  for (const void* p : {io->xb, io->h0, io->h1, io->h2, io->dz2, io->dz1, io->dz0})
    ASVRL_REQUIRE(reinterpret_cast<uintptr_t>(p) % 16 == 0, "asvrl_actor_grads: activations must be 16-byte aligned");
  ASVRL_REQUIRE(reinterpret_cast<uintptr_t>(io->dout) % 8 == 0, "asvrl_actor_grads: dout must be 8-byte aligned");
  return 0;
}

int launch_actor_grads(const AgArgs& a, hipStream_t st) {
  const int blocks = kAgTiles * a.S + kAgOutItems + 1;
  hipLaunchKernelGGL(actor_grads_kernel, dim3(blocks), dim3(kAgT), 0, st, a);
  return check_launch("asvrl_actor_grads");
}
}  // namespace

extern "C" int asvrl_actor_grads(const AsvActorGradIO* io, void* stream) {
  if (int rc = check_actor_grads(io)) return rc;
  if (io->B == 0) return 0;
  AgArgs a{};
  a.io = *io;
  const AgSplit sp = ag_split(io->B);
  a.S = sp.S;
  a.nch = sp.nch;
  return launch_actor_grads(a, as_stream(stream));
}

