// Per-node cost of a chain of dependent kernels replayed from a hipGraph (MI355X), for the
// one-row decode step's launch budget: empty kernels and a kernel whose every block touches
// one cache line, and one with a 384-byte argument block, at 1 / 256 / 2048 blocks of 256
// threads.  Runtime env knobs (HIP_FORCE_DEV_KERNARG, DEBUG_CLR_GRAPH_PACKET_CAPTURE) are
// compared by running it under each (scripts/gpu_launch_env.sh).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void empty_kernel() {}
__global__ void touch_kernel(float* p) {
  if (threadIdx.x == 0) p[blockIdx.x * 16] += 1.0f;
}
// a 384-byte argument block (the size class of GemvArgs / AttnArgs)
struct BigArgs {
  float* p;
  int v[94];
};
__global__ void args_kernel(BigArgs a) {
  if (threadIdx.x == 0) a.p[blockIdx.x * 16] += (float)a.v[blockIdx.x % 94];
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s failed: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

int main() {
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  float* buf = nullptr;
  CK(hipMalloc(&buf, 2048 * 16 * sizeof(float)));
  CK(hipMemset(buf, 0, 2048 * 16 * sizeof(float)));
  const int nodes = 140;
  BigArgs ba{};
  for (int touch = 0; touch < 3; ++touch) {
    for (int blocks : {1, 256, 2048}) {
      hipGraph_t g;
      hipGraphExec_t ge;
      CK(hipStreamBeginCapture(st, hipStreamCaptureModeRelaxed));
      for (int i = 0; i < nodes; ++i) {
        if (touch == 2) { ba.p = buf; ba.v[i % 94] = i; hipLaunchKernelGGL(args_kernel, dim3(blocks), dim3(256), 0, st, ba); }
        else if (touch) hipLaunchKernelGGL(touch_kernel, dim3(blocks), dim3(256), 0, st, buf);
        else hipLaunchKernelGGL(empty_kernel, dim3(blocks), dim3(256), 0, st);
      }
      CK(hipStreamEndCapture(st, &g));
      CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      hipEvent_t e0, e1;
      CK(hipEventCreate(&e0));
      CK(hipEventCreate(&e1));
      for (int w = 0; w < 3; ++w) CK(hipGraphLaunch(ge, st));
      const int reps = 20;
      CK(hipEventRecord(e0, st));
      for (int r = 0; r < reps; ++r) CK(hipGraphLaunch(ge, st));
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      float ms = 0.f;
      CK(hipEventElapsedTime(&ms, e0, e1));
      printf("{\"kernel\": \"%s\", \"blocks\": %d, \"nodes\": %d, \"us_per_node\": %.3f}\n",
             touch == 2 ? "args384" : touch ? "touch" : "empty", blocks, nodes, 1000.f * ms / reps / nodes);
      CK(hipGraphExecDestroy(ge));
      CK(hipGraphDestroy(g));
      CK(hipEventDestroy(e0));
      CK(hipEventDestroy(e1));
    }
  }
  CK(hipFree(buf));
  CK(hipStreamDestroy(st));
  return 0;
}
