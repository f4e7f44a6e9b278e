// Per-kernel cost of a hipGraph replay (diagnostic only): N dependent launches
// of an empty kernel and of a small-grid kernel in one stream, captured once,
// replayed; prints microseconds per launch.  Also the same launches issued
// eagerly.  hipcc -O3 --offload-arch=gfx950 tools/exp/graph_floor.hip -o tools/exp/graph_floor
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__global__ void empty_k(float* p, int n) { if (n < 0) p[threadIdx.x] = 0.f; }
__global__ void touch_k(float* p, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = p[i] * 0.5f + 1.f;
}

int main() {
  float* d;
  CK(hipMalloc(&d, 1 << 24));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  const int N = 200;
  struct Case { const char* name; int grid, blk, n, touch; } cases[] = {
      {"empty_1x64", 1, 64, 0, 0}, {"empty_256x256", 256, 256, 0, 0},
      {"touch_64KB", 64, 256, 1 << 14, 1}, {"touch_4MB", 4096, 256, 1 << 20, 1}};
  for (auto& c : cases) {
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
    for (int i = 0; i < N; ++i) {
      if (c.touch) hipLaunchKernelGGL(touch_k, dim3(c.grid), dim3(c.blk), 0, st, d, c.n);
      else hipLaunchKernelGGL(empty_k, dim3(c.grid), dim3(c.blk), 0, st, d, c.n);
    }
    CK(hipStreamEndCapture(st, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int w = 0; w < 3; ++w) CK(hipGraphLaunch(ge, st));
    CK(hipStreamSynchronize(st));
    CK(hipEventRecord(e0, st));
    for (int r = 0; r < 5; ++r) CK(hipGraphLaunch(ge, st));
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const float graph_us = ms * 1e3f / (5 * N);
    CK(hipEventRecord(e0, st));
    for (int r = 0; r < 5; ++r)
      for (int i = 0; i < N; ++i) {
        if (c.touch) hipLaunchKernelGGL(touch_k, dim3(c.grid), dim3(c.blk), 0, st, d, c.n);
        else hipLaunchKernelGGL(empty_k, dim3(c.grid), dim3(c.blk), 0, st, d, c.n);
      }
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("{\"case\": \"%s\", \"graph_us_per_launch\": %.2f, \"eager_us_per_launch\": %.2f}\n", c.name,
           graph_us, ms * 1e3f / (5 * N));
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
  }
  return 0;
}
