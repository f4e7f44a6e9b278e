// Do parallel branches of a captured hipGraph run concurrently on gfx950?
// (diagnostic only).  Two VALU-spin kernels of G workgroups each, captured
// (a) in one stream, (b) forked onto a second stream and joined with events,
// (c) as one launch of 2G workgroups.  Prints microseconds per replay.
// hipcc -O3 --offload-arch=gfx950 tools/exp/graph_branch.hip -o tools/exp/graph_branch
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__global__ void __launch_bounds__(256) spin_k(float* p, int iters) {
  float a = threadIdx.x * 1e-3f, b = 0.999f;
  for (int i = 0; i < iters; ++i) a = fmaf(a, b, 1e-4f);
  if (a == 12345.f) p[threadIdx.x] = a;
}

static float time_graph(hipGraphExec_t ge, hipStream_t st) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int w = 0; w < 3; ++w) CK(hipGraphLaunch(ge, st));
  CK(hipStreamSynchronize(st));
  CK(hipEventRecord(e0, st));
  for (int r = 0; r < 20; ++r) CK(hipGraphLaunch(ge, st));
  CK(hipEventRecord(e1, st));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms * 1e3f / 20;
}

int main() {
  float* d;
  CK(hipMalloc(&d, 1 << 20));
  hipStream_t st, s2;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  hipEvent_t fork, join;
  CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&join, hipEventDisableTiming));
  const int iters = 4000;
  for (int G : {64, 128}) {
    for (int mode = 0; mode < 4; ++mode) {
      hipGraph_t g;
      hipGraphExec_t ge;
      CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
      for (int rep = 0; rep < 4; ++rep) {
        if (mode == 0) {            // one kernel only (the unit)
          hipLaunchKernelGGL(spin_k, dim3(G), dim3(256), 0, st, d, iters);
        } else if (mode == 1) {     // serial pair
          hipLaunchKernelGGL(spin_k, dim3(G), dim3(256), 0, st, d, iters);
          hipLaunchKernelGGL(spin_k, dim3(G), dim3(256), 0, st, d, iters);
        } else if (mode == 2) {     // forked pair
          CK(hipEventRecord(fork, st));
          CK(hipStreamWaitEvent(s2, fork, 0));
          hipLaunchKernelGGL(spin_k, dim3(G), dim3(256), 0, st, d, iters);
          hipLaunchKernelGGL(spin_k, dim3(G), dim3(256), 0, s2, d, iters);
          CK(hipEventRecord(join, s2));
          CK(hipStreamWaitEvent(st, join, 0));
        } else {                    // one launch of 2G
          hipLaunchKernelGGL(spin_k, dim3(2 * G), dim3(256), 0, st, d, iters);
        }
      }
      CK(hipStreamEndCapture(st, &g));
      CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      const float us = time_graph(ge, st);
      static const char* names[] = {"single", "serial_pair", "forked_pair", "one_launch_2G"};
      printf("{\"G\": %d, \"mode\": \"%s\", \"us_per_rep\": %.2f}\n", G, names[mode], us / 4);
      CK(hipGraphExecDestroy(ge));
      CK(hipGraphDestroy(g));
    }
  }
  return 0;
}
