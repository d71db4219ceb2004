// asvrl_rainbow.hip -- Rainbow's NoisyNet weights and dueling C51 head on gfx950
// (rfarl/rfarl/policy/Rainbow_model.py:17-139, agent.py:308-324,597-641).
//
//   noisy_compose_kernel   W = mu + sigma * eps for every NoisyLinear weight and bias of a network in
//                          one launch (NoisyLinear.forward in training mode, Rainbow_model.py:47-51),
//                          and its backward dmu = dW, dsigma = dW * eps written straight into the
//                          parameters' gradient buffers
//   noisy_reset_kernel     reset_noise() of every layer (Rainbow_model.py:40-45,141-145): factorised
//                          Gaussian noise f(x) = sign(x) sqrt|x| from Philox, eps_w = f(eps_out) f(eps_in)^T,
//                          eps_b = f(eps_out), composed into W in the same launch
//   rainbow_act_kernel     dueling combine q = v + a - mean_a(a), softmax over atoms per action,
//                          Q = sum p z, argmax (first maximum), epsilon-greedy on the device step counter
//                          (act_rainbow, agent.py:308-324; also the double-Q argmax of agent.py:607-609)
//   rainbow_pick_kernel    p(s', a*) of the target net: softmax of q[a*] (agent.py:611-612)
//   rainbow_loss_kernel    loss_b = -sum m log softmax(q[a_b]) (agent.py:633) and the gradient of
//                          mean(w * loss) with respect to the value and advantage logits
//
// The head kernels take the two output layers' logits (f32, rows x 51 and rows x 25*51) from the
// GEMMs; one wave serves two rows, lane = (row, action) for the softmax passes, with the rows'
// advantage logits staged in LDS.
#include "asvrl_common.h"

namespace asvrl {
namespace {

constexpr int kAtoms = 51;
constexpr int kActs = 25;
constexpr int kAdv = kAtoms * kActs;   // 1275
constexpr int kHeadRows = 2;           // rows per wave

// sq_parts (backward, asvrl_noisy_backward_norm): each workgroup's sum of dmu^2 + dsigma^2 in f64, reduced in a
// fixed order (the grid is fixed by the segment total), for the clip norm of the Adam step
__global__ __launch_bounds__(256) void noisy_compose_kernel(AsvNoisySegs s, int backward, double* sq_parts) {
  const int64_t total = s.off[s.n];
  double sq = 0.0;
  for (int64_t g = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; g < total;
       g += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    int k = 0;
    while (g >= s.off[k + 1]) ++k;
    const int64_t i = g - s.off[k];
    const AsvNoisySeg& q = s.seg[k];
    if (!backward) {
      q.out[i] = q.mu[i] + q.sigma[i] * q.eps[i];
    } else {
      const float d = q.dout[i];
      const float ds = d * q.eps[i];
      q.dmu[i] = d;
      q.dsigma[i] = ds;
      sq += static_cast<double>(d) * d + static_cast<double>(ds) * ds;
    }
  }
  if (sq_parts != nullptr) {
    __shared__ double red[256];
    red[threadIdx.x] = sq;
    __syncthreads();
    for (int w = 128; w >= 1; w >>= 1) {
      if (static_cast<int>(threadIdx.x) < w) red[threadIdx.x] += red[threadIdx.x + w];
      __syncthreads();
    }
    if (threadIdx.x == 0) sq_parts[blockIdx.x] = red[0];
  }
}

__device__ __forceinline__ float scale_noise(float x) {   // x.sign() * x.abs().sqrt() (:37-38)
  const float r = __fsqrt_rn(fabsf(x));
  return x > 0.f ? r : (x < 0.f ? -r : 0.f);
}

// reset_noise chunks: each workgroup owns kResetRows output units of one layer (segment pairs: weight 2j,
// bias 2j + 1). The Philox draws are counter-based per (layer, draw index), so every workgroup of a layer
// regenerates the same eps_in and its own eps_out rows; draw j < in is eps_in[j], j >= in is eps_out[j - in].
constexpr int kResetRows = 16;
constexpr int kMaxNoisyLayers = ASVRL_MAX_NOISY_SEGS / 2;
struct NoisyDims {
  int n_layers;
  int in_f[kMaxNoisyLayers], out_f[kMaxNoisyLayers], chunk0[kMaxNoisyLayers + 1];
};

__device__ __forceinline__ float noise_draw(int layer, int j, uint64_t seed, uint64_t ctr) {
  const int t = j >> 1;
  const U4 r = philox4x32_10(U4{static_cast<uint32_t>(t), static_cast<uint32_t>(layer), static_cast<uint32_t>(ctr),
                                static_cast<uint32_t>(ctr >> 32) ^ 0x4E015u},
                             static_cast<uint32_t>(seed), static_cast<uint32_t>(seed >> 32));
  const float u1 = (static_cast<float>(r.x >> 8) + 1.0f) * (1.0f / 16777216.0f);
  const float u2 = static_cast<float>(r.y >> 8) * (1.0f / 16777216.0f);
  const float rad = __fsqrt_rn(-2.0f * __logf(u1));
  float sn, cs;
  __sincosf(6.2831853f * u2, &sn, &cs);
  return scale_noise(rad * ((j & 1) ? sn : cs));   // N(0, 1) -> sign(x) sqrt|x|
}

__global__ __launch_bounds__(256) void noisy_reset_kernel(AsvNoisySegs s, NoisyDims dims, uint64_t seed,
                                                          const int64_t* __restrict__ counter_dev) {
  __shared__ float e_in[256], e_out[kResetRows];
  const int chunk = blockIdx.x;
  int layer = 0;
  while (layer + 1 < dims.n_layers && chunk >= dims.chunk0[layer + 1]) ++layer;
  const int nin = dims.in_f[layer], nout = dims.out_f[layer];
  const int o0 = (chunk - dims.chunk0[layer]) * kResetRows;
  const int no = nout - o0 < kResetRows ? nout - o0 : kResetRows;
  const uint64_t ctr = counter_dev != nullptr ? static_cast<uint64_t>(*counter_dev) : 0ull;
  for (int j = threadIdx.x; j < nin; j += blockDim.x) e_in[j] = noise_draw(layer, j, seed, ctr);
  if (threadIdx.x < no) e_out[threadIdx.x] = noise_draw(layer, nin + o0 + threadIdx.x, seed, ctr);
  __syncthreads();
  const AsvNoisySeg& w = s.seg[2 * layer];
  const AsvNoisySeg& b = s.seg[2 * layer + 1];
  const int n = no * nin;
  const int64_t base = static_cast<int64_t>(o0) * nin;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const int o = i / nin, k = i - o * nin;
    const float e = e_out[o] * e_in[k];   // epsilon_out.ger(epsilon_in) (:44)
    w.eps[base + i] = e;
    w.out[base + i] = w.mu[base + i] + w.sigma[base + i] * e;
  }
  if (threadIdx.x < no) {
    const int o = o0 + threadIdx.x;
    const float e = e_out[threadIdx.x];
    b.eps[o] = e;
    b.out[o] = b.mu[o] + b.sigma[o] * e;
  }
}

// Stage kHeadRows rows of advantage logits (and value logits) in LDS; returns the row base.
struct HeadLds {
  float a[kHeadRows][kAdv];
  float v[kHeadRows][kAtoms + 1];
  float mean[kHeadRows][kAtoms + 1];
};

__device__ __forceinline__ void stage_head(HeadLds& L, const float* __restrict__ v, const float* __restrict__ a,
                                           int64_t ldv, int64_t lda, int row0, int N, int lane) {
#pragma unroll
  for (int r = 0; r < kHeadRows; ++r) {
    const int row = row0 + r;
    if (row < N) {
      for (int i = lane; i < kAdv; i += kWave) L.a[r][i] = a[static_cast<int64_t>(row) * lda + i];
      if (lane < kAtoms) L.v[r][lane] = v[static_cast<int64_t>(row) * ldv + lane];
    }
  }
  __syncthreads();
  // a.mean(1): per (row, atom), the 25 actions in order
#pragma unroll
  for (int r = 0; r < kHeadRows; ++r) {
    if (lane < kAtoms && row0 + r < N) {
      float acc = 0.f;
      for (int k = 0; k < kActs; ++k) acc += L.a[r][k * kAtoms + lane];
      L.mean[r][lane] = acc / static_cast<float>(kActs);
    }
  }
  __syncthreads();
}

// softmax over atoms of q[k] = v + a[k] - mean, then sum p z, one lane per (row, action): online
// max / rescaled sums in one pass over the 51 atoms.
__device__ __forceinline__ float expected_q(const HeadLds& L, int r, int k, const float* __restrict__ z) {
  float mx = -INFINITY, se = 0.f, sz = 0.f;
  for (int i = 0; i < kAtoms; ++i) {
    const float q = L.v[r][i] + L.a[r][k * kAtoms + i] - L.mean[r][i];
    if (q > mx) {
      const float c = __expf(mx - q);
      se = se * c + 1.f;
      sz = sz * c + z[i];
      mx = q;
    } else {
      const float e = __expf(q - mx);
      se += e;
      sz += e * z[i];
    }
  }
  return sz / se;
}

__global__ __launch_bounds__(kWave) void rainbow_act_kernel(AsvRainbowHeadIO io) {
  __shared__ HeadLds L;
  __shared__ float z[kAtoms + 1];
  const int lane = threadIdx.x;
  const int row0 = blockIdx.x * kHeadRows;
  if (lane < kAtoms) z[lane] = io.support[lane];
  stage_head(L, io.v, io.a, io.ldv, io.lda, row0, io.N, lane);
  const int r = lane >> 5, k = lane & 31;
  const int row = row0 + r;
  const bool on = k < kActs && row < io.N;
  float Q = on ? expected_q(L, r, k, z) : -INFINITY;
  int best = on ? k : 1 << 20;
  // argmax within each 32-lane half, first maximum on ties (torch argmax)
#pragma unroll
  for (int off = 16; off > 0; off >>= 1) {
    const float Qo = __shfl_xor(Q, off, kWave);
    const int bo = __shfl_xor(best, off, kWave);
    if (Qo > Q || (Qo == Q && bo < best)) { Q = Qo; best = bo; }
  }
  if (k != 0 || row >= io.N) return;
  double act = static_cast<double>(best);
  if (io.step_dev != nullptr) {
    // epsilon-greedy (agent.py:318-322): greedy iff random() > eps, else a uniform action;
    // eps: linear schedule of the device step counter (trainer.py:257-264)
    const uint64_t step = static_cast<uint64_t>(*io.step_dev);
    const double progress = static_cast<double>(step) * io.eps_steps_per_count / io.eps_total;
    const double eps = progress < io.eps_fraction
                           ? io.eps_initial + (progress / io.eps_fraction) * (io.eps_final - io.eps_initial)
                           : io.eps_final;
    const U4 u = philox4x32_10(U4{static_cast<uint32_t>(row), static_cast<uint32_t>(step),
                                  static_cast<uint32_t>(step >> 32), 0x5A1Bu},
                               static_cast<uint32_t>(io.seed), static_cast<uint32_t>(io.seed >> 32));
    const double c = (static_cast<double>(u.x >> 8) + 1.0) * (1.0 / 16777216.0);   // (0, 1]
    if (!(c > eps)) act = static_cast<double>(u.y % kActs);
  }
  if (io.act_out != nullptr) io.act_out[static_cast<int64_t>(row) * io.ld_act] = act;
  if (io.act_idx != nullptr) io.act_idx[row] = best;
}

// p(s', a*) = softmax(q[a*]) of the target logits, a* from rainbow_act_kernel (act_idx).
__global__ __launch_bounds__(kWave) void rainbow_pick_kernel(AsvRainbowHeadIO io) {
  const int lane = threadIdx.x;
  const int row = blockIdx.x;
  const int64_t* ai = io.act_idx;
  const int k = static_cast<int>(ai[row]);
  const float* a = io.a + static_cast<int64_t>(row) * io.lda;
  float mean = 0.f, q = -INFINITY;
  if (lane < kAtoms) {
    for (int j = 0; j < kActs; ++j) mean += a[j * kAtoms + lane];
    mean /= static_cast<float>(kActs);
    q = io.v[static_cast<int64_t>(row) * io.ldv + lane] + a[k * kAtoms + lane] - mean;
  }
  float mx = q;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) mx = fmaxf(mx, __shfl_xor(mx, off, kWave));
  float e = lane < kAtoms ? __expf(q - mx) : 0.f;
  float se = e;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) se += __shfl_xor(se, off, kWave);
  if (lane < kAtoms) io.p_out[static_cast<int64_t>(row) * kAtoms + lane] = e / se;
}

// loss_b = -sum_i m_i log p_i with p = softmax(q[a_b]); d(mean_b w_b loss_b)/dq_i = (w_b / B)(p_i sum(m) - m_i);
// q[k] = v + a[k] - mean_j a[j] gives dv = dq, da[k] = dq (1{k = a_b} - 1/25).
__global__ __launch_bounds__(kWave) void rainbow_loss_kernel(AsvRainbowHeadIO io) {
  const int lane = threadIdx.x;
  const int row = blockIdx.x;
  const int k = static_cast<int>(io.actions[static_cast<int64_t>(row) * io.ld_rd]);
  const float w = io.weights[static_cast<int64_t>(row) * io.ld_rd];
  const float* a = io.a + static_cast<int64_t>(row) * io.lda;
  float mean = 0.f, q = -INFINITY, m = 0.f;
  if (lane < kAtoms) {
    for (int j = 0; j < kActs; ++j) mean += a[j * kAtoms + lane];
    mean /= static_cast<float>(kActs);
    q = io.v[static_cast<int64_t>(row) * io.ldv + lane] + a[k * kAtoms + lane] - mean;
    m = io.m[static_cast<int64_t>(row) * kAtoms + lane];
  }
  float mx = q;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) mx = fmaxf(mx, __shfl_xor(mx, off, kWave));
  const float e = lane < kAtoms ? expf(q - mx) : 0.f;
  float se = e, sm = m;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    se += __shfl_xor(se, off, kWave);
    sm += __shfl_xor(sm, off, kWave);
  }
  const float lse = mx + logf(se);
  float l = lane < kAtoms ? -m * (q - lse) : 0.f;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) l += __shfl_xor(l, off, kWave);
  if (lane == 0) io.loss[row] = l;
  if (lane >= kAtoms) return;
  const float p = e / se;
  const float dq = (p * sm - m) * w * io.grad_scale;
  io.dv[static_cast<int64_t>(row) * kAtoms + lane] = dq;
  float* da = io.da + static_cast<int64_t>(row) * kAdv;
  const float off_a = -dq / static_cast<float>(kActs);
  for (int j = 0; j < kActs; ++j) da[j * kAtoms + lane] = j == k ? dq + off_a : off_a;
}

int check_segs(const AsvNoisySegs* s, const char* what) {
  ASVRL_REQUIRE(s && s->n >= 1 && s->n <= ASVRL_MAX_NOISY_SEGS, std::string(what) + ": 1..16 segments");
  ASVRL_REQUIRE(s->off[0] == 0, std::string(what) + ": off[0] must be 0");
  for (int k = 0; k < s->n; ++k)
    ASVRL_REQUIRE(s->off[k + 1] >= s->off[k], std::string(what) + ": offsets must be non-decreasing");
  return 0;
}

}  // namespace
}  // namespace asvrl

using namespace asvrl;

namespace {
int noisy_grid(const AsvNoisySegs* segs) {
  const int64_t blocks = (segs->off[segs->n] + 255) / 256;
  return static_cast<int>(blocks < 1024 ? blocks : 1024);
}

int noisy_compose_launch(const AsvNoisySegs* segs, int32_t backward, double* sq_parts, void* stream) {
  if (int rc = check_segs(segs, "asvrl_noisy_compose")) return rc;
  for (int k = 0; k < segs->n; ++k) {
    const AsvNoisySeg& q = segs->seg[k];
    ASVRL_REQUIRE(q.eps && (backward ? (q.dout && q.dmu && q.dsigma) : (q.mu && q.sigma && q.out)),
                  "asvrl_noisy_compose: null segment member");
  }
  if (segs->off[segs->n] == 0) return 0;
  hipLaunchKernelGGL(noisy_compose_kernel, dim3(static_cast<unsigned>(noisy_grid(segs))), dim3(256), 0,
                     as_stream(stream), *segs, backward, sq_parts);
  return check_launch("asvrl_noisy_compose");
}
}  // namespace

extern "C" int asvrl_noisy_compose(const AsvNoisySegs* segs, int32_t backward, void* stream) {
  return noisy_compose_launch(segs, backward, nullptr, stream);
}

extern "C" int32_t asvrl_noisy_backward_norm_parts(const AsvNoisySegs* segs) {
  if (check_segs(segs, "asvrl_noisy_backward_norm_parts") != 0) return 0;
  return segs->off[segs->n] == 0 ? 0 : noisy_grid(segs);
}

extern "C" int asvrl_noisy_backward_norm(const AsvNoisySegs* segs, double* sq_parts, void* stream) {
  ASVRL_REQUIRE(sq_parts != nullptr, "asvrl_noisy_backward_norm: null sq_parts");
  return noisy_compose_launch(segs, 1, sq_parts, stream);
}

extern "C" int asvrl_noisy_reset(const AsvNoisySegs* segs, const int32_t* in_features, const int32_t* out_features,
                                 uint64_t seed, const int64_t* counter_dev, void* stream) {
  if (int rc = check_segs(segs, "asvrl_noisy_reset")) return rc;
  ASVRL_REQUIRE(segs->n % 2 == 0 && in_features && out_features, "asvrl_noisy_reset: (weight, bias) segment pairs");
  NoisyDims d{};
  d.n_layers = segs->n / 2;
  d.chunk0[0] = 0;
  for (int l = 0; l < d.n_layers; ++l) {
    d.in_f[l] = in_features[l];
    d.out_f[l] = out_features[l];
    ASVRL_REQUIRE(d.in_f[l] >= 1 && d.in_f[l] <= 256 && d.out_f[l] >= 1, "asvrl_noisy_reset: in_features in [1, 256]");
    ASVRL_REQUIRE(segs->off[2 * l + 1] - segs->off[2 * l] == static_cast<int64_t>(d.in_f[l]) * d.out_f[l] &&
                      segs->off[2 * l + 2] - segs->off[2 * l + 1] == d.out_f[l],
                  "asvrl_noisy_reset: segment sizes do not match in/out features");
    d.chunk0[l + 1] = d.chunk0[l] + (d.out_f[l] + kResetRows - 1) / kResetRows;
  }
  hipLaunchKernelGGL(noisy_reset_kernel, dim3(d.chunk0[d.n_layers]), dim3(256), 0, as_stream(stream), *segs, d, seed,
                     counter_dev);
  return check_launch("asvrl_noisy_reset");
}

extern "C" int asvrl_rainbow_act(const AsvRainbowHeadIO* io, void* stream) {
  ASVRL_REQUIRE(io && io->v && io->a && io->support && (io->act_out || io->act_idx), "asvrl_rainbow_act: null argument");
  ASVRL_REQUIRE(io->atoms == kAtoms && io->actions_n == kActs, "asvrl_rainbow_act: 51 atoms x 25 actions");
  if (io->N <= 0) return 0;
  hipLaunchKernelGGL(rainbow_act_kernel, dim3((io->N + kHeadRows - 1) / kHeadRows), dim3(kWave), 0,
                     as_stream(stream), *io);
  return check_launch("asvrl_rainbow_act");
}

extern "C" int asvrl_rainbow_pick(const AsvRainbowHeadIO* io, void* stream) {
  ASVRL_REQUIRE(io && io->v && io->a && io->act_idx && io->p_out, "asvrl_rainbow_pick: null argument");
  ASVRL_REQUIRE(io->atoms == kAtoms && io->actions_n == kActs, "asvrl_rainbow_pick: 51 atoms x 25 actions");
  if (io->N <= 0) return 0;
  hipLaunchKernelGGL(rainbow_pick_kernel, dim3(io->N), dim3(kWave), 0, as_stream(stream), *io);
  return check_launch("asvrl_rainbow_pick");
}

extern "C" int asvrl_rainbow_loss(const AsvRainbowHeadIO* io, void* stream) {
  ASVRL_REQUIRE(io && io->v && io->a && io->actions && io->weights && io->m && io->loss && io->dv && io->da,
                "asvrl_rainbow_loss: null argument");
  ASVRL_REQUIRE(io->atoms == kAtoms && io->actions_n == kActs, "asvrl_rainbow_loss: 51 atoms x 25 actions");
  if (io->N <= 0) return 0;
  hipLaunchKernelGGL(rainbow_loss_kernel, dim3(io->N), dim3(kWave), 0, as_stream(stream), *io);
  return check_launch("asvrl_rainbow_loss");
}
