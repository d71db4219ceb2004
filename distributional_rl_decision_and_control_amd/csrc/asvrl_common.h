// asvrl_common.h -- shared device helpers for libasvrl.so (gfx950): error plumbing for the
// C ABI, Philox-4x32-10 counter RNG and the distributions the env draws from.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>

#include "asvrl.h"

namespace asvrl {

constexpr double kPi = 3.141592653589793;   // np.pi
constexpr double kTwoPi = 2 * kPi;           // 2 * np.pi (exact doubling)
constexpr int kWave = 64;                    // CDNA wavefront

void set_error(const std::string& msg);
int check_launch(const char* what);
// out[i] (+)= sum_g partial[g][i] over i < nw (-> dw) and the trailing nb (-> db, optional)
int launch_partial_sum(const float* partial, int groups, int nw, int nb, float* dw, float* db, int accumulate,
                       hipStream_t st);

#define ASVRL_REQUIRE(cond, msg)            \
  do {                                      \
    if (!(cond)) {                          \
      ::asvrl::set_error(std::string(msg)); \
      return 1;                             \
    }                                       \
  } while (0)

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// compute units of the current device (cached; 256 on MI355X when the query fails)
inline int cu_count() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
  }
  return n;
}

// ------------------------------------------------------------------ Philox-4x32-10
struct U4 {
  uint32_t x, y, z, w;
};

__host__ __device__ inline U4 philox4x32_10(U4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = static_cast<uint64_t>(0xD2511F53u) * c.x;
    const uint64_t p1 = static_cast<uint64_t>(0xCD9E8D57u) * c.z;
    const uint32_t h0 = static_cast<uint32_t>(p0 >> 32), l0 = static_cast<uint32_t>(p0);
    const uint32_t h1 = static_cast<uint32_t>(p1 >> 32), l1 = static_cast<uint32_t>(p1);
    c = U4{h1 ^ c.y ^ k0, l1, h0 ^ c.w ^ k1, l0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

// Stream of doubles in (0, 1] from one (key, counter-prefix); each Philox call yields two.
struct Stream {
  uint32_t k0, k1, c1, c2, c3;
  uint32_t n;   // calls made
  U4 buf;
  int left;
  __device__ Stream(uint64_t seed, uint32_t a, uint32_t b, uint32_t c)
      : k0(static_cast<uint32_t>(seed)), k1(static_cast<uint32_t>(seed >> 32)), c1(a), c2(b), c3(c),
        n(0), buf{0, 0, 0, 0}, left(0) {}
  __device__ double u01() {
    if (left == 0) {
      buf = philox4x32_10(U4{n++, c1, c2, c3}, k0, k1);
      left = 2;
    }
    uint64_t hi, lo;
    if (left == 2) { hi = buf.x; lo = buf.y; } else { hi = buf.z; lo = buf.w; }
    --left;
    const uint64_t bits = ((hi << 32) | lo) >> 11;
    return (static_cast<double>(bits) + 1.0) * (1.0 / 9007199254740992.0);
  }
  // Box-Muller pair
  __device__ void normal2(double& a, double& b) {
    const double u1 = u01(), u2 = u01();
    const double rad = sqrt(-2.0 * log(u1));
    double s, c;
    sincos(kTwoPi * u2, &s, &c);
    a = rad * c;
    b = rad * s;
  }
  // von Mises(mu=0, kappa) by Best & Fisher, the algorithm numpy's legacy vonmises uses
  __device__ double vonmises(double kappa) {
    if (kappa < 1e-8) return kPi * (2 * u01() - 1);
    const double r = 1 + sqrt(1 + 4 * kappa * kappa);
    const double rho = (r - sqrt(2 * r)) / (2 * kappa);
    const double s = (1 + rho * rho) / (2 * rho);
    double W = 1.0;
    for (int it = 0; it < 256; ++it) {  // acceptance rate > 0.65 at kappa = 1; bounded loop
      const double U = u01();
      const double Z = cos(kPi * U);
      W = (1 + s * Z) / (s + Z);
      const double Y = kappa * (s - W);
      const double V = u01();
      if ((Y * (2 - Y) - V >= 0) || (log(Y / V) + 1 - Y >= 0)) break;
    }
    const double U = u01();
    double res = acos(W);
    if (U < 0.5) res = -res;
    return res;
  }
};

// f32 draws for the training path (noise_mode 2): the perception noise only has to follow the
// reference's distributions there (N(0, sigma), vonmises(0, kappa), wamv.py:27-40). One Philox call
// (counter 0) feeds the four Gaussians (two Box-Muller pairs); the von Mises radius takes one call per
// two Best-Fisher attempts (counters 1, 2, ...), its sign a spare low bit of the accepted attempt's
// first word (the uniforms use the top 24 bits). No draw indexes a runtime buffer position, so a
// wave whose lanes accept at different attempts issues one Philox call per attempt pair, not per
// draw; the transcendentals, square roots and reciprocals are the single-instruction f32 ones.
struct StreamF {
  uint32_t k0, k1, c1, c2, c3;
  __device__ StreamF(uint64_t seed, uint32_t a, uint32_t b, uint32_t c)
      : k0(static_cast<uint32_t>(seed)), k1(static_cast<uint32_t>(seed >> 32)), c1(a), c2(b), c3(c) {}
  static __device__ float u24(uint32_t w) {   // (0, 1]
    return (static_cast<float>(w >> 8) + 1.0f) * (1.0f / 16777216.0f);
  }
  static __device__ void box_muller(float u1, float u2, float& a, float& b) {
    const float rad = __builtin_amdgcn_sqrtf(-2.0f * __logf(u1));
    const float t = 6.2831853f * u2;
    a = rad * __cosf(t);
    b = rad * __sinf(t);
  }
  __device__ void normal4(float& a, float& b, float& c, float& d) const {
    const U4 w = philox4x32_10(U4{0u, c1, c2, c3}, k0, k1);
    box_muller(u24(w.x), u24(w.y), a, b);
    box_muller(u24(w.z), u24(w.w), c, d);
  }
  // normal4 and, from the same call, a fourth uniform in (0, 1): the low bytes of three of its words (the
  // Gaussians take the top 24 bits of each), for the table-driven von Mises draw (asvrl_env.hip)
  __device__ void normal4u(float& a, float& b, float& c, float& d, float& u) const {
    const U4 w = philox4x32_10(U4{0u, c1, c2, c3}, k0, k1);
    box_muller(u24(w.x), u24(w.y), a, b);
    box_muller(u24(w.z), u24(w.w), c, d);
    const uint32_t spare = ((w.x & 0xFFu) << 16) | ((w.y & 0xFFu) << 8) | (w.z & 0xFFu);
    u = (static_cast<float>(spare) + 0.5f) * (1.0f / 16777216.0f);
  }
  // one Best-Fisher attempt from the uniforms (U, V): W and whether it is accepted
  static __device__ bool attempt(float U, float V, float s, float kappa, float& W) {
    const float Z = __cosf(3.14159265f * U);
    W = (1.0f + s * Z) * __builtin_amdgcn_rcpf(s + Z);
    const float Y = kappa * (s - W);
    return (Y * (2.0f - Y) - V >= 0.0f) || (__logf(Y * __builtin_amdgcn_rcpf(V)) + 1.0f - Y >= 0.0f);
  }
  __device__ float vonmises(float kappa) const {   // Best & Fisher, as Stream::vonmises
    if (kappa < 1e-6f) {
      const U4 w = philox4x32_10(U4{1u, c1, c2, c3}, k0, k1);
      return 3.14159265f * (2.0f * u24(w.x) - 1.0f);
    }
    const float r = 1.0f + __builtin_amdgcn_sqrtf(1.0f + 4.0f * kappa * kappa);
    const float rho = (r - __builtin_amdgcn_sqrtf(2.0f * r)) * __builtin_amdgcn_rcpf(2.0f * kappa);
    const float s = (1.0f + rho * rho) * __builtin_amdgcn_rcpf(2.0f * rho);
    float W = 1.0f;
    uint32_t sgn = 0;
    for (uint32_t blk = 1; blk <= 128; ++blk) {   // acceptance > 0.85 per attempt at kappa = 1; bounded
      const U4 w = philox4x32_10(U4{blk, c1, c2, c3}, k0, k1);
      if (attempt(u24(w.x), u24(w.y), s, kappa, W)) {
        sgn = w.x & 1u;
        break;
      }
      if (attempt(u24(w.z), u24(w.w), s, kappa, W)) {
        sgn = w.z & 1u;
        break;
      }
    }
    const float res = acosf(fminf(fmaxf(W, -1.0f), 1.0f));
    return sgn ? -res : res;
  }
};

// Small-layer weight gradient (f32 dZ, K <= 4 inputs; the action encoder): partial `blk` of 32
// rows, dw[m][k] and db[m] into partial[blk][M*K + M]. Threads 0..255 work, every thread of the
// workgroup must call it (it synchronises); red: 256 x 5 floats of LDS.
constexpr int kSwRows = 32;
__device__ __forceinline__ void small_wgrad_body(const float* __restrict__ dz, int64_t ldz, const float* __restrict__ x,
                                                 int64_t ldx, int R, int M, int K, float* __restrict__ partial,
                                                 int blk, float (*red)[5]) {
  const int t = threadIdx.x;
  const bool act = t < 256;
  const int per = 256 / M;   // rows in flight (M divides 256)
  const int m = t % M, rq = t / M;
  float sw[4] = {0.f, 0.f, 0.f, 0.f}, sb = 0.f;
  const int r0 = blk * kSwRows, r1 = min(R, r0 + kSwRows);
  if (act) {
    for (int r = r0 + rq; r < r1; r += per) {
      const float d = dz[static_cast<int64_t>(r) * ldz + m];
      sb += d;
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (k < K) sw[k] += d * x[static_cast<int64_t>(r) * ldx + k];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) red[t][k] = sw[k];
    red[t][4] = sb;
  }
  __syncthreads();
  if (t < M) {
    float acc[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
    for (int u = t; u < 256; u += M)
#pragma unroll
      for (int k = 0; k < 5; ++k) acc[k] += red[u][k];
    float* p = partial + static_cast<int64_t>(blk) * (M * K + M);
    for (int k = 0; k < K; ++k) p[t * K + k] = acc[k];
    p[M * K + t] = acc[4];
  }
}

// ---------------------------------------------------------------- replay draw (uniform ring)
// The deque position and ring slot of sampled row b (random.sample of replay_buffer.py:26-45, with
// replacement, on Philox(seed, b, ctr)); guard: skip the oldest entries a concurrent push of <= guard
// rows may overwrite. Shared by asvrl_replay_sample and the fused learn prologue (bit-identical draws).
__device__ __forceinline__ int64_t replay_draw_slot(int64_t head, int64_t size, int64_t cap, int64_t guard, int b,
                                                    uint64_t seed, uint64_t ctr) {
  const U4 r = philox4x32_10(U4{static_cast<uint32_t>(b), 0x5A3Bu, static_cast<uint32_t>(ctr >> 32),
                                static_cast<uint32_t>(ctr)},
                             static_cast<uint32_t>(seed), static_cast<uint32_t>(seed >> 32));
  const uint64_t bits = (static_cast<uint64_t>(r.x) << 32) | r.y;
  int64_t lo = size + guard - cap;
  lo = lo > 0 ? lo : 0;
  if (lo >= size) lo = 0;
  const int64_t k = size > 0 ? lo + static_cast<int64_t>(bits % static_cast<uint64_t>(size - lo)) : 0;
  return ((head - size + k) % cap + cap) % cap;   // deque index 0 = oldest
}

// the update's quantile fractions tau ~ U[0, 1) (AC_IQN_model.py:419, torch.rand) of sampled row b:
// tau_sets sets of [B][tau_n], Philox(seed, step) per (row, set, 4 taus), the wave's 64 lanes in turn
__device__ __forceinline__ void replay_draw_taus(int b, int lane, int B, uint64_t seed, uint64_t ctr, float* taus,
                                                 int tau_sets, int tau_n) {
  const int per_row = tau_sets * tau_n;
  for (int k0 = 4 * lane; k0 < per_row; k0 += 4 * kWave) {
    const U4 r = philox4x32_10(U4{static_cast<uint32_t>(b), static_cast<uint32_t>(k0) ^ 0x7A0000u,
                                  static_cast<uint32_t>(ctr >> 32), static_cast<uint32_t>(ctr)},
                               static_cast<uint32_t>(seed) ^ 0x51EDu, static_cast<uint32_t>(seed >> 32));
    const uint32_t w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = k0 + j;
      if (k < per_row) {
        const int set = k / tau_n, t = k - set * tau_n;
        taus[(static_cast<size_t>(set) * B + b) * tau_n + t] = static_cast<float>(w[j] >> 8) * (1.0f / 16777216.0f);
      }
    }
  }
}

// sum of p[k] over k = start, start + step, ... < n in that order, with the loads of each batch of CH
// terms issued before any of them is added (the plain loop waits for every load in turn: one memory round
// trip per term). The same additions in the same order: bit-identical to the plain loop.
template <class T, int CH = 8>
__device__ __forceinline__ T strided_sum(const T* __restrict__ p, int start, int n, int step, T acc) {
  for (int k0 = start; k0 < n; k0 += CH * step) {
    T v[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int k = k0 + c * step;
      v[c] = k < n ? p[k] : T(0);
    }
#pragma unroll
    for (int c = 0; c < CH; ++c)
      if (k0 + c * step < n) acc += v[c];
  }
  return acc;
}

// A kernel's single struct argument read through the kernarg segment pointer (kargs<T>(): the struct must be the
// kernel's first argument) instead of as a by-value parameter, whose fields the compiler loads at kernel entry and
// holds to their last use (spilling SGPRs into VGPR lanes when they outnumber the SGPRs). kfresh() hides the
// pointer's identity, so loads after it are not merged with those before it: a phase or loop iteration that
// re-reads its fields through kfresh(q) holds them for that phase or iteration only (scalar loads, kernarg cache).
template <class T>
using KArg = const __attribute__((address_space(4))) T*;
template <class T>
__device__ __forceinline__ KArg<T> kfresh(KArg<T> q) {
  asm volatile("" : "+s"(q));
  return q;
}
template <class T>
__device__ __forceinline__ const T& kref(KArg<T> q) {
  return *(const T*)q;
}
template <class T>
__device__ __forceinline__ KArg<T> kargs() {
  return (KArg<T>)__builtin_amdgcn_kernarg_segment_ptr();
}

}  // namespace asvrl
