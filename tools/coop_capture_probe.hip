// Probe (not part of the library): can a cooperative launch (grid-wide barrier) be captured into a HIP graph and
// replayed, and what does its grid barrier cost? VERDICT r05 item 4 asked whether the fused critic's 256
// per-workgroup gradient partials could be reduced inside the launch after a grid barrier.
//
//   hipcc --offload-arch=gfx950 -O2 -o oracle/_ref/coop_capture_probe tools/coop_capture_probe.hip
//   ./coop_capture_probe          -> one JSON line
//
// The kernel: every workgroup writes a partial, grid barrier (cooperative_groups grid sync), then workgroup g sums
// slice g of every partial in workgroup order -- the shape the in-launch reduction would have -- on a
// 256-workgroup x 256-thread grid (one workgroup per CU, like the fused critic).
#include <hip/hip_cooperative_groups.h>
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

namespace cg = cooperative_groups;

constexpr int kThreads = 256;

__global__ void coop_kernel(float* parts, float* out, int n_per_group, int reduce) {
  const int g = blockIdx.x, G = gridDim.x;
  for (int i = threadIdx.x; i < n_per_group; i += kThreads) parts[static_cast<size_t>(g) * n_per_group + i] = 1.0f + g;
  if (!reduce) return;
  cg::this_grid().sync();
  const int slice = (n_per_group + G - 1) / G;
  for (int i = g * slice + threadIdx.x; i < (g + 1) * slice && i < n_per_group; i += kThreads) {
    float s = 0.f;
    for (int k = 0; k < G; ++k) s += parts[static_cast<size_t>(k) * n_per_group + i];
    out[i] = s;
  }
}

static const char* err(hipError_t e) { return e == hipSuccess ? "ok" : hipGetErrorString(e); }

int main() {
  int dev = 0, cus = 0, coop = 0;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  hipDeviceGetAttribute(&coop, hipDeviceAttributeCooperativeLaunch, dev);
  const int G = cus, n = 66048;   // the three trunk layers' gradient floats (asvrl_critic_fused.hip)
  float *parts, *out;
  hipMalloc(&parts, sizeof(float) * static_cast<size_t>(G) * n);
  hipMalloc(&out, sizeof(float) * n);
  int reduce = 1;
  void* args[] = {&parts, &out, const_cast<int*>(&n), &reduce};
  hipStream_t s;
  hipStreamCreate(&s);
  // (1) eager cooperative launch, timed
  hipError_t e1 = hipLaunchCooperativeKernel(reinterpret_cast<void*>(coop_kernel), dim3(G), dim3(kThreads), args, 0, s);
  hipStreamSynchronize(s);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipEventRecord(a, s);
  for (int k = 0; k < 20; ++k)
    hipLaunchCooperativeKernel(reinterpret_cast<void*>(coop_kernel), dim3(G), dim3(kThreads), args, 0, s);
  hipEventRecord(b, s);
  hipEventSynchronize(b);
  float ms_coop = 0.f;
  hipEventElapsedTime(&ms_coop, a, b);
  // the same kernel without the barrier and the reduction (partials only), plain launch
  int noreduce = 0;
  void* args0[] = {&parts, &out, const_cast<int*>(&n), &noreduce};
  hipEventRecord(a, s);
  for (int k = 0; k < 20; ++k) hipLaunchKernel(reinterpret_cast<void*>(coop_kernel), dim3(G), dim3(kThreads), args0, 0, s);
  hipEventRecord(b, s);
  hipEventSynchronize(b);
  float ms_plain = 0.f;
  hipEventElapsedTime(&ms_plain, a, b);
  float host = -1.f;
  hipMemcpy(&host, out, sizeof(float), hipMemcpyDeviceToHost);
  // (2) capture into a graph
  hipGraph_t graph = nullptr;
  hipGraphExec_t exec = nullptr;
  hipError_t e_begin = hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
  hipError_t e_launch = hipLaunchCooperativeKernel(reinterpret_cast<void*>(coop_kernel), dim3(G), dim3(kThreads), args, 0, s);
  hipError_t e_end = hipStreamEndCapture(s, &graph);
  hipError_t e_inst = graph ? hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0) : hipErrorInvalidValue;
  hipError_t e_replay = exec ? hipGraphLaunch(exec, s) : hipErrorInvalidValue;
  hipError_t e_sync = hipStreamSynchronize(s);
  hipMemset(out, 0, sizeof(float) * n);
  hipDeviceSynchronize();
  if (exec) {
    hipGraphLaunch(exec, s);
    hipStreamSynchronize(s);
  }
  float host2 = -1.f;
  hipMemcpy(&host2, out, sizeof(float), hipMemcpyDeviceToHost);
  const float expect = static_cast<float>(G) + 0.5f * static_cast<float>(G) * (G - 1);
  std::printf("{\"cus\": %d, \"cooperative_attr\": %d, \"eager_launch\": \"%s\", \"eager_us_per_launch\": %.2f, "
              "\"no_barrier_us_per_launch\": %.2f, \"eager_sum_ok\": %s, \"capture_begin\": \"%s\", "
              "\"capture_launch\": \"%s\", \"capture_end\": \"%s\", \"instantiate\": \"%s\", \"replay\": \"%s\", "
              "\"sync\": \"%s\", \"replay_sum_ok\": %s}\n",
              cus, coop, err(e1), 1e3f * ms_coop / 20, 1e3f * ms_plain / 20, host == expect ? "true" : "false",
              err(e_begin), err(e_launch), err(e_end), err(e_inst), err(e_replay), err(e_sync),
              host2 == expect ? "true" : "false");
  return 0;
}
