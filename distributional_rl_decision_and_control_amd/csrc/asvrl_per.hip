// asvrl_per.hip -- Rainbow's prioritised n-step replay resident in HBM on gfx950
// (ReplayMemory + SegmentTree, rfarl/policy/replay_memory_rainbow.py:14-196).
//
// Layout (AsvPer, include/asvrl.h):
//   rows  [capacity][ASVRL_PER_DIM] f32: obs 40 | action | reward | nonterminal | timestep (i32 bits) | pad 4
//   tree  [2P - 1] f32, P = next pow2 >= capacity: the reference's sum tree with every leaf on the last
//         level (tree_start = P - 1, replay_memory_rainbow.py:17); leaves >= capacity stay 0.
//   Every internal node is f32(left + right) of its children, a pure function of the leaves, so a
//   rebuild of the dirty 2048-leaf blocks plus the top levels reproduces the reference's
//   incremental _propagate / _propagate_index values bit for bit (same pairwise f32 adds).
//
// Deferred mode (the batched trainer). A push of E*R rows at max priority would otherwise put a
// large share of the total mass on the last n time steps, whose windows are incomplete: with
// B = 8192 segments whole segments fall inside that tail and could never be accepted. With
// `deferred` a slot's priority enters the tree only when the push n steps later completes its
// window, so every leaf in the tree is valid and sampling never rejects (the slot at the write
// head still holds complete old data when a sample runs, so the head rule is not needed either).
//
// Streams. One push writes `stride` consecutive slots (one per robot of the env batch), so robot k's
// transitions sit at k, k + stride, k + 2*stride, ...; the n-step window of slot i is
// i, i + stride, ..., i + n*stride. With stride 1 this is exactly the reference's single sequence
// (trainer.py:163-164 appends robots in turn, so there the window spans robots); with stride = the
// batch's robot count each window is one robot's own trajectory. Robots that did not act write a
// blank row (timestep 0, priority 0): never sampled, and it blanks any window that reaches it.
#include "asvrl_common.h"

namespace asvrl {
namespace {

constexpr int kPerDim = ASVRL_PER_DIM;
constexpr int kMeta = ASVRL_OBS_DIM;          // float offset of {action, reward, nonterminal, timestep}
constexpr int kLeafBlock = 2048;              // leaves per subtree workgroup
constexpr int kTreeThreads = 256;
constexpr int kTopThreads = 1024;
constexpr int64_t kMaxLeaves = static_cast<int64_t>(kLeafBlock) * kTopThreads * 2;   // 2^22

__device__ inline int64_t pymod(int64_t a, int64_t m) { return ((a % m) + m) % m; }

// ------------------------------------------------------------------ append (ReplayMemory.append)
// One thread per stream (robot); m = n / stride time slots per call, walked in order (the
// timestep counter t is sequential per stream: t = 0 after a terminal transition,
// replay_memory_rainbow.py:132-139).
__global__ __launch_bounds__(256) void per_push_kernel(const float* __restrict__ obs, const int8_t* __restrict__ cnt,
                                                       const double* __restrict__ actions, int adim,
                                                       const double* __restrict__ reward,
                                                       const uint8_t* __restrict__ done, int n, AsvPer per) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  const int S = per.stride;
  if (r >= S) return;
  const int64_t C = per.capacity;
  const int64_t P = per.tree_leaves;
  const int64_t index = per.state[0];
  const float maxp = per.maxp[0];
  int t = per.t[r];
  for (int k = r; k < n; k += S) {
    const int64_t slot = (index + k) % C;
    float4* dst = reinterpret_cast<float4*>(per.rows + slot * kPerDim);
    const bool valid = cnt[k] >= 0;
    const float prio = valid ? maxp : 0.f;
    if (valid) {
      const float4* src = reinterpret_cast<const float4*>(obs + static_cast<size_t>(k) * ASVRL_OBS_DIM);
#pragma unroll
      for (int q = 0; q < ASVRL_OBS_DIM / 4; ++q) dst[q] = src[q];
      const bool term = done[k] != 0;
      dst[kMeta / 4] = make_float4(static_cast<float>(actions[static_cast<size_t>(k) * adim]),
                                   static_cast<float>(reward[k]), term ? 0.f : 1.f, __int_as_float(t));
      t = term ? 0 : t + 1;
    } else {
      const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int q = 0; q < ASVRL_OBS_DIM / 4; ++q) dst[q] = z;
      dst[kMeta / 4] = z;                  // blank_trans: timestep 0, nonterminal False (:10)
      t = 0;
    }
    // the append priority (max priority, :138) is kept in the slot; without deferral it is the leaf
    dst[kMeta / 4 + 1] = make_float4(prio, 0.f, 0.f, 0.f);
    per.tree[P - 1 + slot] = per.deferred ? 0.f : prio;
    per.dirty[slot / kLeafBlock] = 1;
    if (per.deferred) {
      // the slot whose n-step window this append completes becomes sampleable with the priority it
      // was appended at (a never-written slot holds 0)
      const int64_t act = pymod(index + k - static_cast<int64_t>(per.n_step) * S, C);
      per.tree[P - 1 + act] = per.rows[act * kPerDim + kMeta + 4];
      per.dirty[act / kLeafBlock] = 1;
    }
  }
  per.t[r] = t;
}

// ------------------------------------------------------------------ tree rebuild
// Subtree of one dirty block of Lb leaves: every level in LDS, each node written to its heap slot.
__global__ __launch_bounds__(kTreeThreads) void per_tree_blocks_kernel(float* __restrict__ tree,
                                                                       uint8_t* __restrict__ dirty, int64_t P,
                                                                       int Lb) {
  __shared__ float lv[kLeafBlock];
  const int b = blockIdx.x;
  if (dirty[b] == 0) return;
  const int64_t leaf0 = P - 1 + static_cast<int64_t>(b) * Lb;
  for (int i = threadIdx.x; i < Lb; i += kTreeThreads) lv[i] = tree[leaf0 + i];
  __syncthreads();
  // level with `w` nodes (w = Lb/2 .. 1): depth D - log2(Lb / w); heap index = (Pd - 1) + b*w + i
  int64_t Pd = P >> 1;   // nodes on the level above the leaves
  for (int w = Lb >> 1; w >= 1; w >>= 1, Pd >>= 1) {
    float v[kLeafBlock / kTreeThreads / 2 > 0 ? kLeafBlock / kTreeThreads / 2 : 1];
    int c = 0;
    for (int i = threadIdx.x; i < w; i += kTreeThreads) v[c++] = lv[2 * i] + lv[2 * i + 1];
    __syncthreads();
    c = 0;
    for (int i = threadIdx.x; i < w; i += kTreeThreads) {
      lv[i] = v[c];
      tree[Pd - 1 + static_cast<int64_t>(b) * w + i] = v[c];
      ++c;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) dirty[b] = 0;
}

// Work a push / priority update finishes in its last (one-workgroup) launch instead of launches of their own
// (asvrl_per_push_ex, asvrl_per_update_ex): a device step counter advanced by one, and the mean of the update's
// values in a fixed order.
struct TopExtra {
  int64_t* counter;
  const float* mean_in;
  int mean_n;
  float* mean_out;
};

// The nb block roots up to the root, then the ring advance of a push (and the TopExtra work).
__global__ __launch_bounds__(kTopThreads) void per_tree_top_kernel(float* __restrict__ tree, int nb,
                                                                   int64_t* __restrict__ state, int64_t C,
                                                                   int64_t advance, TopExtra ex) {
  __shared__ float lv[2 * kTopThreads];
  for (int i = threadIdx.x; i < nb; i += kTopThreads) lv[i] = tree[nb - 1 + i];
  __syncthreads();
  for (int w = nb >> 1; w >= 1; w >>= 1) {
    float v0 = 0.f, v1 = 0.f;
    const int i0 = threadIdx.x, i1 = threadIdx.x + kTopThreads;
    if (i0 < w) v0 = lv[2 * i0] + lv[2 * i0 + 1];
    if (i1 < w) v1 = lv[2 * i1] + lv[2 * i1 + 1];
    __syncthreads();
    if (i0 < w) { lv[i0] = v0; tree[w - 1 + i0] = v0; }
    if (i1 < w) { lv[i1] = v1; tree[w - 1 + i1] = v1; }
    __syncthreads();
  }
  if (threadIdx.x == 0 && advance != 0) {
    const int64_t nx = state[0] + advance;
    if (nx >= C) state[1] = 1;           // full = full or index == 0 after a wrap (:147)
    state[0] = nx % C;
  }
  if (threadIdx.x == 0 && ex.counter != nullptr) ex.counter[0] += 1;
  if (ex.mean_out != nullptr) {   // thread t sums values t, t + 1024, ... in order, then a fixed pairwise tree
    float v = 0.f;
    for (int i = threadIdx.x; i < ex.mean_n; i += kTopThreads) v += ex.mean_in[i];
    __syncthreads();
    lv[threadIdx.x] = v;
    __syncthreads();
    for (int w = kTopThreads >> 1; w >= 1; w >>= 1) {
      if (threadIdx.x < w) lv[threadIdx.x] += lv[threadIdx.x + w];
      __syncthreads();
    }
    if (threadIdx.x == 0) ex.mean_out[0] = lv[0] / static_cast<float>(ex.mean_n);
  }
}

// weights / weights.max() (replay_memory_rainbow.py:191) over the sampled rows' weight column, in place: one
// workgroup (the max is order-independent, the quotient IEEE: the values of torch's w.div_(w.max())). It reads the
// weights from the contiguous copy asvrl_per_sample_ex wrote beside the rows (coalesced; the rows' column is one
// float per 352-byte row), kNormPer per thread in flight and kept in registers for the quotients.
constexpr int kNormPer = 8;
__global__ __launch_bounds__(kTopThreads) void per_normalise_kernel(float* __restrict__ rows,
                                                                    const float* __restrict__ wsrc, int B) {
  __shared__ float mx[kTopThreads];
  float m = -__builtin_inff();
  float v[kNormPer];
  for (int b0 = 0; b0 < B; b0 += kTopThreads * kNormPer) {
#pragma unroll
    for (int j = 0; j < kNormPer; ++j) {   // every load of the chunk issued before the first use
      const int b = b0 + j * kTopThreads + static_cast<int>(threadIdx.x);
      v[j] = b < B ? wsrc[b] : -__builtin_inff();
    }
#pragma unroll
    for (int j = 0; j < kNormPer; ++j) m = fmaxf(m, v[j]);
  }
  mx[threadIdx.x] = m;
  __syncthreads();
  for (int w = kTopThreads >> 1; w >= 1; w >>= 1) {
    if (threadIdx.x < w) mx[threadIdx.x] = fmaxf(mx[threadIdx.x], mx[threadIdx.x + w]);
    __syncthreads();
  }
  const float d = mx[0];
  if (B <= kTopThreads * kNormPer) {   // the one chunk is still in registers
#pragma unroll
    for (int j = 0; j < kNormPer; ++j) {
      const int b = j * kTopThreads + static_cast<int>(threadIdx.x);
      if (b < B) rows[static_cast<int64_t>(b) * ASVRL_TR_DIM + 84] = v[j] / d;
    }
    return;
  }
  for (int b = threadIdx.x; b < B; b += kTopThreads) rows[static_cast<int64_t>(b) * ASVRL_TR_DIM + 84] = wsrc[b] / d;
}

// ------------------------------------------------------------------ sample (ReplayMemory.sample)
// One thread per segment: stratified value, descent in f64 against the f32 nodes exactly as
// SegmentTree._retrieve (:72-84), validity test of _get_samples_from_segments (:159-165) with a
// per-segment Philox redraw (the segments are independent, so redrawing only a rejected segment
// has the distribution of the reference's redraw of the whole batch), then the n-step window
// (:143-154) and the importance weight before batch-max normalisation (:190-191).
__global__ __launch_bounds__(256) void per_sample_kernel(AsvPer per, int B, const double* __restrict__ uniforms,
                                                         uint64_t seed, uint64_t counter,
                                                         const uint64_t* __restrict__ counter_dev,
                                                         float* __restrict__ out, int64_t* __restrict__ out_idx,
                                                         float* __restrict__ w_out) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const int64_t C = per.capacity, P = per.tree_leaves;
  const int S = per.stride, n = per.n_step;
  const int64_t index = per.state[0];
  const bool full = per.state[1] != 0;
  const float total = per.tree[0];
  const float seg = total / static_cast<float>(B);              // p_total / batch_size (f32)
  const double segd = static_cast<double>(seg);
  const double start = static_cast<double>(b) * segd;           // np.arange(B) * segment_length (f64)
  const uint64_t ctr = counter + (counter_dev != nullptr ? *counter_dev : 0ull);
  int64_t node = 0;
  float prob = 0.f;
  int64_t di = 0;
  bool ok = false;
  const int attempts = uniforms != nullptr ? 1 : 64;
  for (int a = 0; a < attempts && !ok; ++a) {
    double u;
    if (uniforms != nullptr) {
      u = uniforms[b];
    } else {
      const U4 r = philox4x32_10(U4{static_cast<uint32_t>(b), 0x9E11u + static_cast<uint32_t>(a),
                                    static_cast<uint32_t>(ctr >> 32), static_cast<uint32_t>(ctr)},
                                 static_cast<uint32_t>(seed), static_cast<uint32_t>(seed >> 32));
      const uint64_t bits = ((static_cast<uint64_t>(r.x) << 32) | r.y) >> 11;
      u = static_cast<double>(bits) * (1.0 / 9007199254740992.0);          // [0, 1)
    }
    double val = (0.0 + segd * u) + start;   // np.random.uniform(0, seg) + segment_starts
    node = 0;
    while (node < P - 1) {
      const int64_t l = 2 * node + 1;
      const double lv = static_cast<double>(per.tree[l]);
      if (val > lv) {
        val -= lv;
        node = l + 1;
      } else {
        node = l;
      }
    }
    if (node > P - 1 + C - 1) node = P - 1 + C - 1;   // children clipped to the last leaf (:78-79)
    prob = per.tree[node];
    di = node - (P - 1);
    if (per.deferred)   // distance behind the head in [1, C]: the head slot is the oldest complete data
      ok = pymod(index - di - 1, C) + 1 > static_cast<int64_t>(n) * S && prob != 0.f;
    else                // :163
      ok = pymod(index - di, C) > static_cast<int64_t>(n) * S && pymod(di - index, C) >= S && prob != 0.f;
  }
  if (!ok) atomicAdd(reinterpret_cast<unsigned long long*>(per.state + 3), 1ull);   // reported, row still valid data
  // an unvalidated draw's leaf is marked -1: update_priorities skips it (the reference never updates a
  // draw it did not accept; a priority written there could make an empty slot sampleable)
  out_idx[b] = ok ? node : -1;
  // n-step window: blank from the first later transition whose timestep is 0 (:146-150)
  float rew[8];
  bool blank = false;
  float nonterm = 0.f;
  int64_t last = di;
  for (int m = 0; m <= n; ++m) {
    const int64_t s = (di + static_cast<int64_t>(m) * S) % C;
    const float4 meta = reinterpret_cast<const float4*>(per.rows + s * kPerDim)[kMeta / 4];
    if (m > 0) blank = blank || __float_as_int(meta.w) == 0;
    if (m < n) rew[m] = blank ? 0.f : meta.y;
    if (m == n) nonterm = blank ? 0.f : meta.z;
    last = s;
  }
  const float* r0 = per.rows + di * kPerDim;
  float4* o = reinterpret_cast<float4*>(out + static_cast<size_t>(b) * ASVRL_TR_DIM);
#pragma unroll
  for (int q = 0; q < ASVRL_OBS_DIM / 4; ++q) o[q] = reinterpret_cast<const float4*>(r0)[q];
  const float4* rn = reinterpret_cast<const float4*>(per.rows + last * kPerDim);
#pragma unroll
  for (int q = 0; q < ASVRL_OBS_DIM / 4; ++q) o[ASVRL_OBS_DIM / 4 + q] = blank ? make_float4(0.f, 0.f, 0.f, 0.f) : rn[q];
  // R = rewards @ n_step_scaling (:179-180), scaling[k] = f32(discount ** k)
  float R = 0.f;
  double sc = 1.0;
  for (int m = 0; m < n; ++m) {
    R += rew[m] * static_cast<float>(sc);
    sc *= per.discount;
  }
  const float p = prob / total;                                            // probs / p_total
  const int64_t cap = full ? C : index;
  // (capacity * probs) ** -beta; a draw that never validated (64 rejected redraws, counted above) gets
  // weight 0 -- it may sit on a zero-priority leaf, where the power is inf and w / w.max() would turn
  // the whole batch NaN -- so it takes no part in the loss
  const float w = ok ? powf(static_cast<float>(cap) * p, -per.priority_weight) : 0.f;
  o[2 * ASVRL_OBS_DIM / 4] = make_float4(r0[kMeta], 0.f, R, nonterm);
  o[2 * ASVRL_OBS_DIM / 4 + 1] = make_float4(w, p, static_cast<float>(di), 0.f);
  if (w_out != nullptr) w_out[b] = w;   // the contiguous copy asvrl_per_normalise reads
}

// ------------------------------------------------------------------ update_priorities
// values ** priority_exponent (exponent 0.5: correctly rounded sqrt), written to the sampled leaves.
// The stratified draws come out in non-decreasing leaf order, so duplicates are adjacent and the
// last one wins as in numpy's fancy assignment (:50); the running max (:52-53) by atomicMax on the
// bit pattern (non-negative floats order like their bits).
__global__ __launch_bounds__(256) void per_update_kernel(AsvPer per, const int64_t* __restrict__ tree_idx,
                                                         const float* __restrict__ values, int B, int raw) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  float v = 0.f;
  if (i < B) {
    const float x = values[i];
    v = raw ? x : (per.priority_exponent == 0.5f ? __fsqrt_rn(x) : powf(x, per.priority_exponent));
    const int64_t ti = tree_idx[i];
    // the next VALID draw's leaf (-1 marks an unvalidated draw, asvrl_per_sample): duplicates are
    // adjacent among the valid ones
    int64_t nx = -1;
    for (int j = i + 1; j < B && nx < 0; ++j) nx = tree_idx[j];
    const bool last = nx != ti;
    if (ti >= 0 && nx >= 0 && nx < ti) atomicAdd(reinterpret_cast<unsigned long long*>(per.state + 3), 1ull);
    if (ti < 0) v = 0.f;   // skipped: no write, no part in the running max
    if (ti >= 0 && last) {
      per.tree[ti] = v;
      per.dirty[(ti - (per.tree_leaves - 1)) / kLeafBlock] = 1;
    }
  }
  float m = v;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off, kWave));
  if ((threadIdx.x & 63) == 0 && i - static_cast<int>(threadIdx.x & 63) < B)
    atomicMax(reinterpret_cast<int*>(per.maxp), __float_as_int(m));
}

int launch_rebuild(const AsvPer& per, int64_t advance, hipStream_t st, const char* what, const TopExtra& ex = {}) {
  const int64_t P = per.tree_leaves;
  const int Lb = static_cast<int>(P < kLeafBlock ? P : kLeafBlock);
  const int nb = static_cast<int>(P / Lb);
  if (Lb > 1) {
    hipLaunchKernelGGL(per_tree_blocks_kernel, dim3(nb), dim3(kTreeThreads), 0, st, per.tree, per.dirty, P, Lb);
    if (int rc = check_launch(what)) return rc;
  }
  hipLaunchKernelGGL(per_tree_top_kernel, dim3(1), dim3(kTopThreads), 0, st, per.tree, nb, per.state,
                     per.capacity, advance, ex);
  return check_launch(what);
}

int check_per(const AsvPer* per, const char* what) {
  ASVRL_REQUIRE(per && per->rows && per->tree && per->state && per->t && per->maxp && per->dirty,
                std::string(what) + ": null AsvPer member");
  const int64_t P = per->tree_leaves;
  ASVRL_REQUIRE(P >= 2 && (P & (P - 1)) == 0 && P <= kMaxLeaves,
                std::string(what) + ": tree_leaves must be a power of two in [2, 2^22]");
  ASVRL_REQUIRE(per->capacity >= 2 && per->capacity <= P && P < 2 * per->capacity,
                std::string(what) + ": tree_leaves must be the next power of two >= capacity");
  ASVRL_REQUIRE(per->stride >= 1 && per->capacity % per->stride == 0,
                std::string(what) + ": capacity must be a multiple of stride");
  ASVRL_REQUIRE(per->n_step >= 1 && per->n_step <= 8, std::string(what) + ": n_step in [1, 8]");
  ASVRL_REQUIRE(static_cast<int64_t>(per->n_step + 2) * per->stride <= per->capacity,
                std::string(what) + ": capacity too small for the n-step window");
  return 0;
}

}  // namespace
}  // namespace asvrl

using namespace asvrl;

extern "C" int asvrl_per_push_ex(const AsvPer* per, const float* obs, const int8_t* obj_cnt, const double* actions,
                                 int32_t action_dim, const double* reward, const uint8_t* done, int32_t n,
                                 int64_t* step_counter, void* stream) {
  if (int rc = check_per(per, "asvrl_per_push")) return rc;
  ASVRL_REQUIRE(obs && obj_cnt && actions && reward && done, "asvrl_per_push: null argument");
  ASVRL_REQUIRE(action_dim >= 1, "asvrl_per_push: action_dim >= 1");
  ASVRL_REQUIRE(n >= 0 && n % per->stride == 0 && n <= per->capacity,
                "asvrl_per_push: n must be a multiple of stride and <= capacity");
  if (n == 0) return 0;
  const hipStream_t st = as_stream(stream);
  hipLaunchKernelGGL(per_push_kernel, dim3((per->stride + 255) / 256), dim3(256), 0, st, obs, obj_cnt, actions,
                     action_dim, reward, done, n, *per);
  if (int rc = check_launch("asvrl_per_push")) return rc;
  TopExtra ex{};
  ex.counter = step_counter;
  return launch_rebuild(*per, n, st, "asvrl_per_push(tree)", ex);
}

extern "C" int asvrl_per_push(const AsvPer* per, const float* obs, const int8_t* obj_cnt, const double* actions,
                              int32_t action_dim, const double* reward, const uint8_t* done, int32_t n,
                              void* stream) {
  return asvrl_per_push_ex(per, obs, obj_cnt, actions, action_dim, reward, done, n, nullptr, stream);
}

extern "C" int asvrl_per_sample_ex(const AsvPer* per, int32_t B, const double* uniforms, uint64_t seed,
                                   uint64_t counter, const uint64_t* counter_dev, float* out, int64_t* out_tree_idx,
                                   float* weights, void* stream) {
  if (int rc = check_per(per, "asvrl_per_sample")) return rc;
  ASVRL_REQUIRE(out && out_tree_idx, "asvrl_per_sample: null argument");
  ASVRL_REQUIRE(B >= 1, "asvrl_per_sample: B >= 1");
  hipLaunchKernelGGL(per_sample_kernel, dim3((B + 255) / 256), dim3(256), 0, as_stream(stream), *per, B, uniforms,
                     seed, counter, counter_dev, out, out_tree_idx, weights);
  return check_launch("asvrl_per_sample");
}

extern "C" int asvrl_per_sample(const AsvPer* per, int32_t B, const double* uniforms, uint64_t seed,
                                uint64_t counter, const uint64_t* counter_dev, float* out, int64_t* out_tree_idx,
                                void* stream) {
  return asvrl_per_sample_ex(per, B, uniforms, seed, counter, counter_dev, out, out_tree_idx, nullptr, stream);
}

extern "C" int asvrl_per_update_ex(const AsvPer* per, const int64_t* tree_idx, const float* values, int32_t B,
                                   int32_t raw, float* values_mean, int64_t* learn_counter, void* stream) {
  if (int rc = check_per(per, "asvrl_per_update")) return rc;
  ASVRL_REQUIRE(tree_idx && values, "asvrl_per_update: null argument");
  if (B <= 0) return 0;
  const hipStream_t st = as_stream(stream);
  hipLaunchKernelGGL(per_update_kernel, dim3((B + 255) / 256), dim3(256), 0, st, *per, tree_idx, values, B, raw);
  if (int rc = check_launch("asvrl_per_update")) return rc;
  TopExtra ex{};
  ex.counter = learn_counter;
  ex.mean_in = values;
  ex.mean_n = B;
  ex.mean_out = values_mean;
  return launch_rebuild(*per, 0, st, "asvrl_per_update(tree)", ex);
}

extern "C" int asvrl_per_update(const AsvPer* per, const int64_t* tree_idx, const float* values, int32_t B,
                                int32_t raw, void* stream) {
  return asvrl_per_update_ex(per, tree_idx, values, B, raw, nullptr, nullptr, stream);
}

extern "C" int asvrl_per_normalise(float* rows, const float* weights, int32_t B, void* stream) {
  ASVRL_REQUIRE(rows != nullptr && weights != nullptr && B >= 1, "asvrl_per_normalise: null argument or B < 1");
  hipLaunchKernelGGL(per_normalise_kernel, dim3(1), dim3(kTopThreads), 0, as_stream(stream), rows, weights, B);
  return check_launch("asvrl_per_normalise");
}
