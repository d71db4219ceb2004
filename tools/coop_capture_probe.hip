// Probe (not part of the library): can a cooperative launch (grid-wide barrier) be captured into a HIP graph and
// replayed, and what would an in-launch reduction of the fused critic's per-workgroup gradient partials cost?
// VERDICT r05 item 4 asked whether the 256 partials could be reduced inside the launch after a grid barrier.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/coop_capture_probe tools/coop_capture_probe.hip
//   ./coop_capture_probe          -> one JSON line
//
// Shape of the fused critic (asvrl_critic_fused.hip): 256 workgroups x 256 threads (one per CU), each writes its
// 66,048-float partial (the three trunk layers' dW + db), then
//   mode 0  nothing more (plain launch): the partial stores alone
//   mode 1  + the cooperative grid barrier: the barrier's cost
//   mode 2  + the reduction after the barrier: workgroup g sums slice g of every partial in workgroup order
//           (deterministic), each wave a quarter of the partials with 16 loads in flight per lane, the four
//           waves' sums added in wave order through LDS
//   split   mode 0 followed by a separate reduction launch of the same arithmetic on 1,032 workgroups of 64
//           outputs each (partial_sums_kernel's kind of shape)
// Round 6's first version of this probe reduced with one dependent load per partial (185 us); it said nothing
// about the barrier. Times: HIP events over 20 back-to-back launches.
#include <hip/hip_cooperative_groups.h>
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>

namespace cg = cooperative_groups;

constexpr int kThreads = 256, kN = 66048, kInFlight = 16;

__device__ __forceinline__ void write_partial(float* parts, int g) {
  float4* p = reinterpret_cast<float4*>(parts + static_cast<size_t>(g) * kN);
  for (int i = threadIdx.x; i < kN / 4; i += kThreads) {
    const float v = 1.0f + static_cast<float>(g) + 1e-3f * static_cast<float>(i & 7);
    p[i] = make_float4(v, v, v, v);
  }
}

// outputs o0 .. o0 + 63 (lane), partials k0 .. k0 + nk - 1 (in order), kInFlight loads issued before the adds
__device__ __forceinline__ float sum_parts(const float* parts, int o, int k0, int nk) {
  float s = 0.f;
  for (int k = k0; k < k0 + nk; k += kInFlight) {
    float v[kInFlight];
#pragma unroll
    for (int j = 0; j < kInFlight; ++j) v[j] = o < kN ? parts[static_cast<size_t>(k + j) * kN + o] : 0.f;
#pragma unroll
    for (int j = 0; j < kInFlight; ++j) s += v[j];
  }
  return s;
}

// workgroup-wide: outputs [lo, hi) in chunks of 64, wave w sums partials w G/4 .. (w + 1) G/4 - 1, the four
// wave sums added in wave order
__device__ __forceinline__ void reduce_slice(const float* parts, float* out, int lo, int hi, int G) {
  __shared__ float ws[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, q = G / 4;
  for (int c = lo; c < hi; c += 64) {
    const int o = c + lane;
    ws[w][lane] = sum_parts(parts, o < hi ? o : kN, w * q, q);
    __syncthreads();
    if (w == 0 && o < hi) out[o] = ((ws[0][lane] + ws[1][lane]) + ws[2][lane]) + ws[3][lane];
    __syncthreads();
  }
}

__global__ __launch_bounds__(kThreads) void coop_kernel(float* parts, float* out, int mode) {
  const int g = blockIdx.x, G = gridDim.x;
  write_partial(parts, g);
  if (mode == 0) return;
  cg::this_grid().sync();
  if (mode == 1) return;
  const int slice = (kN + G - 1) / G;
  const int lo = g * slice, hi = lo + slice < kN ? lo + slice : kN;
  reduce_slice(parts, out, lo, hi, G);
}

// the separate reduction: 64 outputs per workgroup (4 waves), G partials
__global__ __launch_bounds__(kThreads) void reduce_kernel(const float* parts, float* out, int G) {
  const int lo = blockIdx.x * 64, hi = lo + 64 < kN ? lo + 64 : kN;
  reduce_slice(parts, out, lo, hi, G);
}

static const char* err(hipError_t e) { return e == hipSuccess ? "ok" : hipGetErrorString(e); }

int main() {
  int dev = 0, cus = 0, coop = 0;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  hipDeviceGetAttribute(&coop, hipDeviceAttributeCooperativeLaunch, dev);
  int G = cus;
  if (G % (4 * kInFlight) != 0) G = G / (4 * kInFlight) * (4 * kInFlight);   // a quarter per wave, 16 per batch
  float *parts, *out;
  hipMalloc(&parts, sizeof(float) * static_cast<size_t>(G) * kN);
  hipMalloc(&out, sizeof(float) * kN);
  hipStream_t s;
  hipStreamCreate(&s);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  constexpr int kReps = 20;
  float us[3] = {0.f, 0.f, 0.f};
  hipError_t e_mode[3];
  for (int mode = 0; mode < 3; ++mode) {
    int m = mode;
    void* args[] = {&parts, &out, &m};
    e_mode[mode] = hipLaunchCooperativeKernel(reinterpret_cast<void*>(coop_kernel), dim3(G), dim3(kThreads), args, 0, s);
    hipStreamSynchronize(s);
    hipEventRecord(a, s);
    for (int k = 0; k < kReps; ++k)
      hipLaunchCooperativeKernel(reinterpret_cast<void*>(coop_kernel), dim3(G), dim3(kThreads), args, 0, s);
    hipEventRecord(b, s);
    hipEventSynchronize(b);
    float ms = 0.f;
    hipEventElapsedTime(&ms, a, b);
    us[mode] = 1e3f * ms / kReps;
  }
  // expected sum of output o: sum_g (1 + g + 1e-3 (o & 7)) in f32 over the same order is not reproducible on the
  // host bit for bit; check to 1e-4 relative
  auto check = [&](bool& ok) {
    static float host[kN];
    hipMemcpy(host, out, sizeof(host), hipMemcpyDeviceToHost);
    ok = true;
    for (int o = 0; o < kN; o += 997) {
      double e = 0.0;
      for (int g = 0; g < G; ++g) e += 1.0 + g + 1e-3 * ((o / 4) & 7);
      if (std::fabs(host[o] - e) > 1e-4 * e) ok = false;
    }
  };
  bool ok_coop = false;
  check(ok_coop);
  // plain partial launch + separate reduction launch
  hipMemset(out, 0, sizeof(float) * kN);
  int m0 = 0;
  hipEventRecord(a, s);
  for (int k = 0; k < kReps; ++k) {
    hipLaunchKernelGGL(coop_kernel, dim3(G), dim3(kThreads), 0, s, parts, out, m0);
    hipLaunchKernelGGL(reduce_kernel, dim3((kN + 63) / 64), dim3(kThreads), 0, s, parts, out, G);
  }
  hipEventRecord(b, s);
  hipEventSynchronize(b);
  float ms_split = 0.f;
  hipEventElapsedTime(&ms_split, a, b);
  bool ok_split = false;
  check(ok_split);
  // capture of the cooperative launch (mode 2) into a graph, replayed
  int m2 = 2;
  void* args2[] = {&parts, &out, &m2};
  hipGraph_t graph = nullptr;
  hipGraphExec_t exec = nullptr;
  hipError_t e_begin = hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
  hipError_t e_launch = hipLaunchCooperativeKernel(reinterpret_cast<void*>(coop_kernel), dim3(G), dim3(kThreads), args2, 0, s);
  hipError_t e_end = hipStreamEndCapture(s, &graph);
  hipError_t e_inst = graph ? hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0) : hipErrorInvalidValue;
  hipMemset(out, 0, sizeof(float) * kN);
  hipDeviceSynchronize();
  hipError_t e_replay = exec ? hipGraphLaunch(exec, s) : hipErrorInvalidValue;
  hipError_t e_sync = hipStreamSynchronize(s);
  bool ok_replay = false;
  check(ok_replay);
  std::printf("{\"cus\": %d, \"workgroups\": %d, \"partial_floats\": %d, \"cooperative_attr\": %d, "
              "\"launch\": [\"%s\", \"%s\", \"%s\"], \"us_partials_only\": %.2f, \"us_partials_grid_barrier\": %.2f, "
              "\"us_partials_barrier_inlaunch_reduce\": %.2f, \"us_partials_then_reduce_launch\": %.2f, "
              "\"inlaunch_sum_ok\": %s, \"split_sum_ok\": %s, \"capture\": [\"%s\", \"%s\", \"%s\", \"%s\"], "
              "\"replay\": \"%s\", \"sync\": \"%s\", \"replay_sum_ok\": %s}\n",
              cus, G, kN, coop, err(e_mode[0]), err(e_mode[1]), err(e_mode[2]), us[0], us[1], us[2],
              1e3f * ms_split / kReps, ok_coop ? "true" : "false", ok_split ? "true" : "false", err(e_begin),
              err(e_launch), err(e_end), err(e_inst), err(e_replay), err(e_sync), ok_replay ? "true" : "false");
  return 0;
}
