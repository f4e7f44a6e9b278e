// What makes a captured kernel node cost more than the 1.6 us floor
// (diagnostic only): N launches per graph of
//   small   12-byte kernarg, empty body
//   big     1 KB kernarg struct passed by value (read: one field), empty body
//   lds     small kernarg, 32 KB dynamic LDS
//   code10  ten distinct kernels with ~24 KB of unrolled code each, cycled
//   bigrd   1 KB kernarg, every thread reads 64 fields of it
// Prints microseconds per launch (graph replay).
//   hipcc -O3 --offload-arch=gfx950 tools/exp/graph_floor2.hip -o tools/exp/graph_floor2
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

struct Big { float* p; int n; int pad[254]; };
__global__ void small_k(float* p, int n) { if (n < 0) p[threadIdx.x] = 0.f; }
__global__ void big_k(Big a) { if (a.n < 0) a.p[threadIdx.x] = 0.f; }
__global__ void bigrd_k(Big a) {
  int s = 0;
#pragma unroll
  for (int i = 0; i < 64; ++i) s += a.pad[i * 3];
  if (s == 12345 && a.n < 0) a.p[threadIdx.x] = 0.f;
}
__global__ void lds_k(float* p, int n) {
  extern __shared__ float sm[];
  if (n < 0) { sm[threadIdx.x] = 1.f; p[threadIdx.x] = sm[threadIdx.x ^ 1]; }
}
template <int K>
__global__ void code_k(float* p, int n) {
  float x = threadIdx.x * 1.0001f + K;
  if (n < 0) {
#pragma unroll
    for (int i = 0; i < 1500; ++i) x = x * 1.0000001f + (float)(i ^ K);
    p[threadIdx.x] = x;
  }
}
typedef void (*CF)(float*, int);
CF codes[10] = {code_k<0>, code_k<1>, code_k<2>, code_k<3>, code_k<4>,
                code_k<5>, code_k<6>, code_k<7>, code_k<8>, code_k<9>};

int main() {
  float* d;
  CK(hipMalloc(&d, 1 << 20));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  CK(hipFuncSetAttribute((const void*)lds_k, hipFuncAttributeMaxDynamicSharedMemorySize, 32768));
  const int N = 200;
  Big big{};
  big.p = d;
  big.n = 1;
  const char* names[5] = {"small", "big", "lds", "code10", "bigrd"};
  for (int c = 0; c < 5; ++c) {
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
    for (int i = 0; i < N; ++i) {
      if (c == 0) hipLaunchKernelGGL(small_k, dim3(64), dim3(256), 0, st, d, 1);
      else if (c == 1) hipLaunchKernelGGL(big_k, dim3(64), dim3(256), 0, st, big);
      else if (c == 2) hipLaunchKernelGGL(lds_k, dim3(64), dim3(256), 32768, st, d, 1);
      else if (c == 3) hipLaunchKernelGGL(codes[i % 10], dim3(64), dim3(256), 0, st, d, 1);
      else hipLaunchKernelGGL(bigrd_k, dim3(64), dim3(256), 0, st, big);
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
    printf("{\"case\": \"%s\", \"graph_us_per_launch\": %.2f}\n", names[c], ms * 1e3f / (5 * N));
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
  }
  return 0;
}
