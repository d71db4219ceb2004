// asvrl_learn.hip -- learner-side kernels of the rfarl hot path on gfx950:
//   * the fused quantile-Huber loss + gradient (agent.py:406-412, 701-707),
//   * the C51 categorical projection (agent.py:616-631), bit-exact to the CPU reference,
//   * the replay ring (ReplayBuffer.add/sample, replay_buffer.py:22-69) resident in HBM,
// plus the ABI's error plumbing.
#include "asvrl_common.h"

namespace asvrl {

thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

int check_launch(const char* what) {
  const hipError_t err = hipGetLastError();
  if (err != hipSuccess) {
    set_error(std::string(what) + ": " + hipGetErrorString(err));
    return 2;
  }
  return 0;
}

namespace {

__device__ inline float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
  return v;
}

// ------------------------------------------------------------------ quantile Huber
// One wave per batch row: lane i owns expected quantile qe[b,i] (i = lane, lane+64, ...)
// and sweeps the Np target quantiles, which are wave-uniform loads.
constexpr int kQhWaves = 4;

__global__ __launch_bounds__(kQhWaves * kWave) void quantile_huber_kernel(
    const float* __restrict__ qt, const float* __restrict__ qe, const float* __restrict__ tau, int B,
    int N, int Np, float kappa, float gscale, float* __restrict__ row_loss, float* __restrict__ dqe) {
  const int lane = threadIdx.x & (kWave - 1);
  const int b = blockIdx.x * kQhWaves + (threadIdx.x >> 6);
  if (b >= B) return;
  const float* qtb = qt + static_cast<size_t>(b) * Np;
  float part = 0.f;
  for (int i0 = 0; i0 < N; i0 += kWave) {
    const int i = i0 + lane;
    if (i < N) {
      const float e = qe[static_cast<size_t>(b) * N + i];
      const float t = tau[static_cast<size_t>(b) * N + i];
      float acc_l = 0.f, acc_g = 0.f;
      for (int j = 0; j < Np; ++j) {
        const float d = qtb[j] - e;  // td_error = Q_targets - Q_expected (agent.py:406)
        const float ad = fabsf(d);
        const bool quad = ad <= kappa;
        const float h = quad ? 0.5f * (d * d) : kappa * (ad - 0.5f * kappa);
        const float w = fabsf(t - (d < 0.f ? 1.f : 0.f));  // |tau - 1{td < 0}| (agent.py:409)
        acc_l += w * h / kappa;
        acc_g += w * (quad ? d : (d > 0.f ? kappa : -kappa)) / kappa;
      }
      part += acc_l;
      dqe[static_cast<size_t>(b) * N + i] = -acc_g * gscale;
    }
  }
  part = wave_sum(part);
  if (lane == 0) row_loss[b] = part / static_cast<float>(Np);
}

__global__ __launch_bounds__(1024) void mean_kernel(const float* __restrict__ x, int n, float* __restrict__ out) {
  __shared__ float sh[1024 / kWave];
  float v = 0.f;
  for (int k = threadIdx.x; k < n; k += blockDim.x) v += x[k];
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x < kWave) {
    float w = threadIdx.x < (blockDim.x >> 6) ? sh[threadIdx.x] : 0.f;
    w = wave_sum(w);
    if (threadIdx.x == 0) out[0] = w / static_cast<float>(n);
  }
}

// ------------------------------------------------------------------ C51 projection
// One wave per row, lane j = atom j. The reference accumulates with two sequential CPU index_add_
// passes (lower masses, then upper masses, each in atom order), so m[k] = ((0 + the lower masses with
// l_j = k, in j order) + the upper masses with u_j = k, in j order). b_j is non-decreasing in j
// (Tz = R + nonterminal * gamma^n * z_j with nonterminal * gamma^n >= 0, clamp and the affine map are
// monotone under rounding), and so are l_j and u_j after the two integer fixes, so the j with a
// given l (or u) form one contiguous run. Each lane finds whether it starts / ends its target's run from
// its neighbours' targets (DPP wave shifts, no LDS), records the bounds in LDS at the target's slot, and
// lane k then adds exactly its own runs in order: bit-identical to the reference.
//
// Each wave owns its LDS slices and handles ROWS rows whose loads are all issued before the first
// projection; the LDS hand-offs are wave-local (a wave's LDS instructions execute in order, so only the
// compiler has to be kept from reordering them -- no workgroup barrier). Round 3: one row per wave and
// three workgroup barriers per row, 5.8 us at B = 8192 (0.074 of HBM), 26 us at B = 65536.
//
// Round 4: the serial part batched across rows. A run is at most two atoms long unless atoms clamp at
// Vmin / Vmax or the row is terminal (b_{j+1} - b_j = gamma^n * nonterminal <= 1); the round-3 kernel walked
// every long run on the whole wave, one row after another (up to 2 x 51 dependent adds per row: 23 us at
// B = 65536, 0.147 of HBM). Now a wave stages its ROWS rows in LDS (masses and each target's run bounds
// as four bytes), finishes every target whose runs are short with selects (one ds_read2 per pass), and
// queues the others as (row, target) jobs that the wave's lanes then walk in parallel, one job per lane.
// The run bounds are scattered by masked byte stores (only the lanes that bound a run write); the row's
// scalars come through the scalar cache. Same additions in the same order: bit-identical.
constexpr int kC51Waves = 4;
#ifndef ASVRL_C51_ROWS
#define ASVRL_C51_ROWS 4
#endif
// the workgroup's long-run jobs pooled and walked by its first waves (1), or each wave its own (0): at
// four rows per wave 16.8 -> 15.9 us at B = 65536; at two (B = 8192) 5.5 -> 5.9 us, so there each wave its own
// (profiles/r04aa_c51_pool_ab.txt)
#ifndef ASVRL_C51_POOL
#define ASVRL_C51_POOL 1
#endif

// acc + v[j0] + v[j0+1] + ... + v[j1-1], added in order; the LDS reads go out 8 at a time
__device__ __forceinline__ float run_sum(const float* v, int j0, int j1, float acc) {
  int j = j0;
  for (; j + 8 <= j1; j += 8) {
    float x[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) x[k] = v[j + k];
#pragma unroll
    for (int k = 0; k < 8; ++k) acc += x[k];
  }
  for (; j < j1; ++j) acc += v[j];
  return acc;
}

// the wave's own LDS stores before this point are ordered before its LDS reads after it (compiler only:
// the hardware executes one wave's LDS instructions in order)
__device__ __forceinline__ void wave_lds_order() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// lane - 1's / lane + 1's value (DPP wave_shr:1 / wave_shl:1); `edge` where there is no such lane
__device__ __forceinline__ int from_prev_lane(int v, int edge) { return __builtin_amdgcn_update_dpp(edge, v, 0x138, 0xF, 0xF, false); }
__device__ __forceinline__ int from_next_lane(int v, int edge) { return __builtin_amdgcn_update_dpp(edge, v, 0x130, 0xF, 0xF, false); }

template <int ROWS>
__global__ __launch_bounds__(kC51Waves * kWave) void c51_kernel(const float* __restrict__ pns_a,
                                                                const float* __restrict__ ret, int64_t ld_ret,
                                                                const float* __restrict__ nonterm, int64_t ld_nt,
                                                                const float* __restrict__ support, int B,
                                                                int atoms, float vmin, float vmax, float dz,
                                                                float gamma_n, float* __restrict__ m) {
  // per wave and row: the lower / upper masses (a 65th slot for the second read of a run starting at lane
  // 63) and per target its runs' bounds as bytes {lower start, lower end, upper start, upper end}; the
  // workgroup's long-run jobs ((wave * ROWS + row) << 6 | target), walked by the first waves after a barrier
  // (kPool: ASVRL_C51_POOL at four rows per wave; else each wave walks its own)
  __shared__ float s_lo[kC51Waves][ROWS][kWave + 1], s_up[kC51Waves][ROWS][kWave + 1];
  __shared__ uint32_t s_rb[kC51Waves][ROWS][kWave + 1];
  __shared__ uint16_t s_job[kC51Waves * ROWS * kWave];
  __shared__ int s_njob;
  constexpr bool kPool = ASVRL_C51_POOL && ROWS >= 4;
  const int lane = threadIdx.x & (kWave - 1);
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int row0 = (blockIdx.x * kC51Waves + w) * ROWS;
  const int nr = B - row0 < ROWS ? (B - row0 > 0 ? B - row0 : 0) : ROWS;   // wave-uniform
  const bool lane_on = lane < atoms;
  const float z = lane_on ? support[lane] : 0.f;
  float pv[ROWS], rv[ROWS], nv[ROWS];
#pragma unroll
  for (int r = 0; r < ROWS; ++r) {
    const int b = row0 + r;
    const bool on = r < nr && lane_on;
    pv[r] = on ? __builtin_nontemporal_load(pns_a + static_cast<size_t>(b) * atoms + lane) : 0.f;
    rv[r] = r < nr ? ret[b * ld_ret] : 0.f;
    nv[r] = r < nr ? nonterm[b * ld_nt] : 0.f;
  }
  if (kPool && threadIdx.x == 0) s_njob = 0;
  // (1) every row's masses into LDS, bounds cleared; targets and run-boundary flags kept in registers
  int lt[ROWS], ut[ROWS];
  uint32_t fl[ROWS];
#pragma unroll
  for (int r = 0; r < ROWS; ++r) {
    const float ntg = nv[r] * gamma_n;
    float tz = rv[r] + ntg * z;                   // Tz = R + nonterminal * gamma^n * z
    tz = fminf(fmaxf(tz, vmin), vmax);            // clamp(Vmin, Vmax)
    const float bb = (tz - vmin) / dz;            // b = (Tz - Vmin) / delta_z
    int l = static_cast<int>(floorf(bb));
    int u = static_cast<int>(ceilf(bb));
    if (u > 0 && l == u) l -= 1;                  // agent.py:623
    if (l < atoms - 1 && l == u) u += 1;          // agent.py:624
    s_lo[w][r][lane] = pv[r] * (static_cast<float>(u) - bb);
    s_up[w][r][lane] = pv[r] * (bb - static_cast<float>(l));
    s_rb[w][r][lane] = 0u;
    const bool on = lane_on && r < nr;
    if (!on) l = u = -1;
    // off lanes carry target -1, lane 0 sees -2 before it: a valid target (>= 0) differs from both
    const int lp = from_prev_lane(l, -2), ln = from_next_lane(l, -2);
    const int up = from_prev_lane(u, -2), un = from_next_lane(u, -2);
    lt[r] = l;
    ut[r] = u;
    fl[r] = (on && lp != l ? 1u : 0u) | (on && ln != l ? 2u : 0u) | (on && up != u ? 4u : 0u) | (on && un != u ? 8u : 0u);
  }
  if (lane == 0) {
#pragma unroll
    for (int r = 0; r < ROWS; ++r) s_lo[w][r][kWave] = s_up[w][r][kWave] = 0.f;
  }
  wave_lds_order();
  // (2) run bounds: the first / last lane of each run writes its target's byte
#pragma unroll
  for (int r = 0; r < ROWS; ++r) {
    unsigned char* rb = reinterpret_cast<unsigned char*>(&s_rb[w][r][0]);
    // masked stores: the lanes bounding no run would all hit one dummy address (a 64-way bank conflict)
    if (fl[r] & 1u) rb[4 * lt[r] + 0] = static_cast<unsigned char>(lane);
    if (fl[r] & 2u) rb[4 * lt[r] + 1] = static_cast<unsigned char>(lane + 1);
    if (fl[r] & 4u) rb[4 * ut[r] + 2] = static_cast<unsigned char>(lane);
    if (fl[r] & 8u) rb[4 * ut[r] + 3] = static_cast<unsigned char>(lane + 1);
  }
  wave_lds_order();
  if constexpr (kPool) __syncthreads();   // s_njob's initial value before any wave appends
  // (3) lane k = target k: short runs finished with selects, long ones queued
  int njob = 0;
#pragma unroll
  for (int r = 0; r < ROWS; ++r) {
    if (r >= nr) break;   // wave-uniform
    const uint32_t q = s_rb[w][r][lane];
    const int ls = q & 255u, ll = static_cast<int>((q >> 8) & 255u) - ls;
    const int us = (q >> 16) & 255u, ul = static_cast<int>(q >> 24) - us;
    const float a0 = s_lo[w][r][ls], a1 = s_lo[w][r][ls + 1];
    const float c0 = s_up[w][r][us], c1 = s_up[w][r][us + 1];
    float acc = 0.f;
    acc = ll > 0 ? acc + a0 : acc;
    acc = ll > 1 ? acc + a1 : acc;
    acc = ul > 0 ? acc + c0 : acc;
    acc = ul > 1 ? acc + c1 : acc;
    const bool lng = ll > 2 || ul > 2;
    if (lane_on && !lng) __builtin_nontemporal_store(acc, m + static_cast<size_t>(row0 + r) * atoms + lane);
    const unsigned long long jm = __ballot(lng);
    if (jm != 0ull) {
      const int before = __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(jm >> 32),
                                                   __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(jm), 0u));
      int base = njob;
      if constexpr (kPool) {
        int b0 = 0;
        if (lane == 0) b0 = atomicAdd(&s_njob, __popcll(jm));
        base = __builtin_amdgcn_readfirstlane(b0);
      }
      if (lng) s_job[(kPool ? 0 : w * ROWS * kWave) + base + before] = static_cast<uint16_t>(((w * ROWS + r) << 6) | lane);
      njob += __popcll(jm);
    }
  }
  if constexpr (kPool) {
    __syncthreads();
    njob = s_njob;
  } else {
    if (njob == 0) return;   // wave-uniform
    wave_lds_order();
  }
  // (4) the long runs, one (row, target) per lane, each summed in order
  const uint16_t* jobs = s_job + (kPool ? 0 : w * ROWS * kWave);
  for (int j0 = kPool ? w * kWave : 0; j0 < njob; j0 += (kPool ? kC51Waves : 1) * kWave) {
    if (j0 + lane < njob) {
      const int job = jobs[j0 + lane];
      const int wr = job >> 6, k = job & 63;
      const int jw = wr / ROWS, r = wr % ROWS;
      const uint32_t q = s_rb[jw][r][k];
      float acc = run_sum(&s_lo[jw][r][0], q & 255u, (q >> 8) & 255u, 0.f);
      acc = run_sum(&s_up[jw][r][0], (q >> 16) & 255u, q >> 24, acc);
      const int grow = (blockIdx.x * kC51Waves + jw) * ROWS + r;
      __builtin_nontemporal_store(acc, m + static_cast<size_t>(grow) * atoms + k);
    }
  }
}

// ------------------------------------------------------------------ replay ring
constexpr int kPushBlock = 256;
// the last block takes the push's row count from the blocks' own counts (one integer atomic each) instead of
// recounting every flag: IQN loop 0.2947 -> 0.2930 ms, AC-IQN unchanged (profiles/r04ad_push_sumcount_ab.txt)

__device__ __forceinline__ int block_sum(int v, int* sh) {
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  int t = 0;
  for (int w = 0; w < kPushBlock / kWave; ++w) t += sh[w];
  return t;
}

// rows of cnt[0, lim) that push (obj_cnt >= 0), counted by the whole block: sixteen flags per 16-byte
// load when cnt is 16-byte aligned, the loads of a thread issued together (the flags are L2-resident:
// the count costs a few L2 round trips, not one per 4 KB)
__device__ __forceinline__ int sign_bytes(uint32_t w) { return __popc(w & 0x80808080u); }
__device__ __forceinline__ int count_pushed(const int8_t* __restrict__ cnt, int lim, int* sh) {
  int c = 0;
  int done = 0;
  if ((reinterpret_cast<uintptr_t>(cnt) & 15) == 0) {
    const uint4* c16 = reinterpret_cast<const uint4*>(cnt);
    const int n16 = lim / 16;
#pragma unroll 8
    for (int q = threadIdx.x; q < n16; q += kPushBlock) {
      const uint4 v = c16[q];
      c += 16 - (sign_bytes(v.x) + sign_bytes(v.y) + sign_bytes(v.z) + sign_bytes(v.w));
    }
    done = n16 * 16;
  }
  for (int k = done + threadIdx.x; k < lim; k += kPushBlock) c += cnt[k] >= 0 ? 1 : 0;
  return block_sum(c, sh);
}

// ReplayBuffer.add for every robot that acted (trainer.py:163-166) in ONE launch: block b's first slot
// follows the rows of the earlier blocks that push (counted by the block itself from the L2-resident
// flags: the row order of the deque, deterministic); the last block to arrive (a counter it resets)
// advances {head, size} and, when asked, copies the new state to `snap` (the ring snapshot the next learn
// step samples against) and increments `counter_inc` (the env step counter).
__global__ __launch_bounds__(kPushBlock) void replay_push_kernel(
    const float* __restrict__ obs_prev, const float* __restrict__ obs_next, const int8_t* __restrict__ cnt,
    const double* __restrict__ actions, int adim, int64_t ald, const double* __restrict__ reward,
    const uint8_t* __restrict__ done, int n, float* __restrict__ ring, int64_t cap, int64_t* ring_state,
    int* arrive, int nblocks, int64_t* snap, int64_t* counter_inc) {
  __shared__ int sh[kPushBlock / kWave], shw[kPushBlock / kWave];
  __shared__ int s_last;
  __shared__ int64_t s_slot[kPushBlock];   // the ring slot of each of the block's rows, -1: not pushed
  const int before = count_pushed(cnt, static_cast<int>(blockIdx.x) * kPushBlock, sh);
  const int k = blockIdx.x * kPushBlock + threadIdx.x;
  const bool v = k < n && cnt[k] >= 0;
  const unsigned long long bal = __ballot(v);
  const int lane = threadIdx.x & 63;
  const int rank_in_wave = __popcll(bal & ((1ull << lane) - 1ull));
  if (lane == 0) shw[threadIdx.x >> 6] = __popcll(bal);
  __syncthreads();
  const int64_t head_in = ring_state[0];
  if (v) {
    int wave_off = 0;
    for (int w = 0; w < (threadIdx.x >> 6); ++w) wave_off += shw[w];
    const int64_t slot = (head_in + before + wave_off + rank_in_wave) % cap;
    float4* dst = reinterpret_cast<float4*>(ring + slot * ASVRL_TR_DIM);
    s_slot[threadIdx.x] = slot;
    const float a0 = static_cast<float>(actions[k * ald]);
    const float a1 = adim > 1 ? static_cast<float>(actions[k * ald + 1]) : 0.f;
    dst[2 * ASVRL_OBS_DIM / 4] = make_float4(a0, a1, static_cast<float>(reward[k]), done[k] ? 1.f : 0.f);
    dst[2 * ASVRL_OBS_DIM / 4 + 1] = make_float4(0.f, 0.f, 0.f, 0.f);
  } else {
    s_slot[threadIdx.x] = -1;
  }
  __syncthreads();
  {   // the block's observation rows copied cooperatively: thread t moves 16-byte pieces t, t + 256, ... so a
      // wave's loads and stores cover whole row runs, not one piece of 64 rows 352 B apart (push 29.8 -> 21.6 us
      // in the step, profiles/r05am_push_coalesced_ab.txt)
    constexpr int kQ = ASVRL_OBS_DIM / 4;   // 16-byte pieces per observation row
    const int k0 = blockIdx.x * kPushBlock;
    const int nr = n - k0 < kPushBlock ? n - k0 : kPushBlock;
    const float4* a4 = reinterpret_cast<const float4*>(obs_prev) + static_cast<size_t>(k0) * kQ;
    const float4* b4 = reinterpret_cast<const float4*>(obs_next) + static_cast<size_t>(k0) * kQ;
#pragma unroll 10
    for (int q = threadIdx.x; q < nr * kQ; q += kPushBlock) {
      const int r = q / kQ;
      const float4 x = a4[q], y = b4[q];   // in bounds for every row of the block: loads ahead of the test
      const int64_t slot = s_slot[r];
      if (slot >= 0) {
        float4* dst = reinterpret_cast<float4*>(ring + slot * ASVRL_TR_DIM) + (q - r * kQ);
        dst[0] = x;
        dst[kQ] = y;
      }
    }
  }
  __syncthreads();   // every lane's read of ring_state is done before the block arrives
  if (threadIdx.x == 0) {
    int cb = 0;
    for (int w = 0; w < kPushBlock / kWave; ++w) cb += shw[w];
    atomicAdd(arrive + 1, cb);   // the push's row count, block by block (integers: the order does not matter)
    __threadfence();
    s_last = atomicAdd(arrive, 1) == nblocks - 1;
  }
  __syncthreads();
  if (!s_last) return;
  if (threadIdx.x == 0) {
    const int tot = atomicExch(arrive + 1, 0);   // every block's count (added before its arrival), reset
    const int64_t nh = (head_in + tot) % cap, ns0 = ring_state[1] + tot;
    const int64_t ns = ns0 < cap ? ns0 : cap;
    ring_state[0] = nh;
    ring_state[1] = ns;
    if (snap != nullptr) {
      snap[0] = nh;
      snap[1] = ns;
    }
    if (counter_inc != nullptr) *counter_inc += 1;
    *arrive = 0;
  }
}

// one wave per sampled row, 22 lanes x float4
__global__ __launch_bounds__(4 * kWave) void replay_sample_kernel(const float* __restrict__ ring, int64_t cap,
                                                                  const int64_t* __restrict__ ring_state,
                                                                  const int64_t* __restrict__ indices, int B,
                                                                  uint64_t seed, uint64_t counter,
                                                                  const uint64_t* __restrict__ counter_dev,
                                                                  int64_t guard, float* __restrict__ out,
                                                                  int64_t* out_slots, float* __restrict__ taus,
                                                                  int tau_sets, int tau_n) {
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;
  const int64_t head = ring_state[0];
  const int64_t size = ring_state[1];
  const uint64_t ctr = counter + (counter_dev != nullptr ? *counter_dev : 0ull);
  const int64_t slot = indices != nullptr ? ((head - size + indices[b]) % cap + cap) % cap
                                          : replay_draw_slot(head, size, cap, guard, b, seed, ctr);
  if (lane == 0 && out_slots != nullptr) out_slots[b] = slot;
  if (taus != nullptr) replay_draw_taus(b, lane, B, seed, ctr, taus, tau_sets, tau_n);
  if (lane < ASVRL_TR_DIM / 4) {
    const float4* src = reinterpret_cast<const float4*>(ring + slot * ASVRL_TR_DIM);
    reinterpret_cast<float4*>(out + static_cast<size_t>(b) * ASVRL_TR_DIM)[lane] = src[lane];
  }
}

__global__ __launch_bounds__(4 * kWave) void replay_write_rows_kernel(const float* __restrict__ rows,
                                                                      const int64_t* __restrict__ slots, int n,
                                                                      float* __restrict__ ring) {
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= n || lane >= ASVRL_TR_DIM / 4) return;
  reinterpret_cast<float4*>(ring + slots[b] * ASVRL_TR_DIM)[lane] =
      reinterpret_cast<const float4*>(rows + static_cast<size_t>(b) * ASVRL_TR_DIM)[lane];
}

}  // namespace
}  // namespace asvrl

using namespace asvrl;

extern "C" const char* asvrl_last_error(void) { return g_last_error.c_str(); }
extern "C" int asvrl_abi_version(void) { return ASVRL_ABI_VERSION; }
extern "C" void asvrl_struct_sizes(int64_t* out5) {
  out5[0] = sizeof(AsvParams);
  out5[1] = sizeof(AsvEnvState);
  out5[2] = sizeof(AsvStepCtl);
  out5[3] = sizeof(AsvStepOut);
  out5[4] = sizeof(AsvResetCfg);
}

extern "C" int asvrl_quantile_huber(const float* qt, const float* qe, const float* tau, int32_t B, int32_t N,
                                    int32_t Np, float kappa, float grad_scale, float* row_loss, float* loss,
                                    float* dqe, void* stream) {
  ASVRL_REQUIRE(qt && qe && tau && row_loss && dqe, "asvrl_quantile_huber: null argument");
  ASVRL_REQUIRE(B >= 0 && N >= 1 && Np >= 1 && kappa > 0.f, "asvrl_quantile_huber: bad shape/kappa");
  if (B == 0) return 0;
  const float gscale = grad_scale / (static_cast<float>(B) * static_cast<float>(Np));
  hipLaunchKernelGGL(quantile_huber_kernel, dim3((B + kQhWaves - 1) / kQhWaves), dim3(kQhWaves * kWave), 0,
                     as_stream(stream), qt, qe, tau, B, N, Np, kappa, gscale, row_loss, dqe);
  if (int rc = check_launch("asvrl_quantile_huber")) return rc;
  if (loss != nullptr) {
    hipLaunchKernelGGL(mean_kernel, dim3(1), dim3(1024), 0, as_stream(stream), row_loss, B, loss);
    return check_launch("asvrl_quantile_huber(mean)");
  }
  return 0;
}

extern "C" int asvrl_c51_project_ex(const float* pns_a, const float* returns, int64_t ld_ret,
                                    const float* nonterminal, int64_t ld_nt, const float* support, int32_t B,
                                    int32_t atoms, float vmin, float vmax, float delta_z, float gamma_n, float* m,
                                    void* stream) {
  ASVRL_REQUIRE(pns_a && returns && nonterminal && support && m, "asvrl_c51_project: null argument");
  ASVRL_REQUIRE(atoms >= 2 && atoms <= kWave, "asvrl_c51_project: atoms must be in [2, 64]");
  ASVRL_REQUIRE(ld_ret >= 1 && ld_nt >= 1, "asvrl_c51_project: strides must be positive");
  if (B <= 0) return 0;
  // rows per wave: one below 4096 rows (latency: every row its own wave), two below 32768, else
  // ASVRL_C51_ROWS (their loads in flight together, their long runs walked side by side)
  auto go = [&](auto kern, int rows) {
    hipLaunchKernelGGL(kern, dim3((B + kC51Waves * rows - 1) / (kC51Waves * rows)), dim3(kC51Waves * kWave), 0,
                       as_stream(stream), pns_a, returns, ld_ret, nonterminal, ld_nt, support, B, atoms, vmin, vmax,
                       delta_z, gamma_n, m);
  };
  if (B < 4096)
    go(c51_kernel<1>, 1);
  else if (B < 32768)
    go(c51_kernel<2>, 2);
  else
    go(c51_kernel<ASVRL_C51_ROWS>, ASVRL_C51_ROWS);
  return check_launch("asvrl_c51_project");
}

extern "C" int asvrl_c51_project(const float* pns_a, const float* returns, const float* nonterminal,
                                 const float* support, int32_t B, int32_t atoms, float vmin, float vmax,
                                 float delta_z, float gamma_n, float* m, void* stream) {
  return asvrl_c51_project_ex(pns_a, returns, 1, nonterminal, 1, support, B, atoms, vmin, vmax, delta_z, gamma_n, m,
                              stream);
}

extern "C" int asvrl_replay_push_ex(const float* obs_prev, const float* obs_next, const int8_t* obj_cnt_next,
                                    const double* actions, int32_t action_dim, int64_t action_ld,
                                    const double* reward,
                                    const uint8_t* done, int32_t n, float* ring, int64_t capacity,
                                    int64_t* ring_state, int32_t* work, int64_t* snap, int64_t* counter_inc,
                                    void* stream) {
  ASVRL_REQUIRE(obs_prev && obs_next && obj_cnt_next && actions && reward && done && ring && ring_state && work,
                "asvrl_replay_push: null argument");
  ASVRL_REQUIRE(capacity >= n && capacity > 0, "asvrl_replay_push: capacity smaller than one push");
  ASVRL_REQUIRE(action_dim == 1 || action_dim == 2, "asvrl_replay_push: action_dim must be 1 or 2");
  ASVRL_REQUIRE(action_ld >= action_dim, "asvrl_replay_push: action row stride below action_dim");
  if (n <= 0) return 0;
  const int nb = (n + kPushBlock - 1) / kPushBlock;
  hipLaunchKernelGGL(replay_push_kernel, dim3(nb), dim3(kPushBlock), 0, as_stream(stream), obs_prev, obs_next,
                     obj_cnt_next, actions, action_dim, action_ld, reward, done, n, ring, capacity, ring_state, work, nb, snap,
                     counter_inc);
  return check_launch("asvrl_replay_push");
}

extern "C" int asvrl_replay_push(const float* obs_prev, const float* obs_next, const int8_t* obj_cnt_next,
                                 const double* actions, int32_t action_dim, const double* reward,
                                 const uint8_t* done, int32_t n, float* ring, int64_t capacity,
                                 int64_t* ring_state, int32_t* work, void* stream) {
  return asvrl_replay_push_ex(obs_prev, obs_next, obj_cnt_next, actions, action_dim, action_dim, reward, done, n, ring, capacity,
                              ring_state, work, nullptr, nullptr, stream);
}

extern "C" int asvrl_replay_sample(const float* ring, int64_t capacity, const int64_t* ring_state,
                                   const int64_t* indices, int32_t B, uint64_t seed, uint64_t counter,
                                   const uint64_t* counter_dev, int64_t guard, float* out, int64_t* out_slots,
                                   float* taus, int32_t tau_sets, int32_t tau_n, void* stream) {
  ASVRL_REQUIRE(ring && ring_state && out, "asvrl_replay_sample: null argument");
  ASVRL_REQUIRE(capacity > 0, "asvrl_replay_sample: bad capacity");
  ASVRL_REQUIRE(taus == nullptr || (tau_sets >= 1 && tau_n >= 1), "asvrl_replay_sample: bad tau shape");
  if (B <= 0) return 0;
  hipLaunchKernelGGL(replay_sample_kernel, dim3((B + 3) / 4), dim3(4 * kWave), 0, as_stream(stream), ring,
                     capacity, ring_state, indices, B, seed, counter, counter_dev, guard, out, out_slots, taus,
                     tau_sets, tau_n);
  return check_launch("asvrl_replay_sample");
}

extern "C" int asvrl_replay_write_rows(const float* rows, const int64_t* slots, int32_t n, float* ring,
                                       void* stream) {
  ASVRL_REQUIRE(rows && slots && ring, "asvrl_replay_write_rows: null argument");
  if (n <= 0) return 0;
  hipLaunchKernelGGL(replay_write_rows_kernel, dim3((n + 3) / 4), dim3(4 * kWave), 0, as_stream(stream), rows,
                     slots, n, ring);
  return check_launch("asvrl_replay_write_rows");
}
