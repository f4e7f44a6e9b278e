// Developer experiment (not part of the library): HBM ceilings for the GAE
// byte mix.  Build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC -o tools/exp/libgae_exp.so tools/exp/gae_exp.hip
#include <hip/hip_runtime.h>
#include <stdint.h>

// read three float4 streams, write two (the GAE mix), grid-stride, U in flight
__global__ void __launch_bounds__(256) exp_stream(const float4* __restrict__ a, const float4* __restrict__ b,
                                                  const float4* __restrict__ c, int64_t na4, int64_t nc4,
                                                  float4* __restrict__ o1, float4* __restrict__ o2,
                                                  int64_t no4, float* sink) {
  const int64_t tid = (int64_t)blockIdx.x * 256 + threadIdx.x, nth = (int64_t)gridDim.x * 256;
  float acc = 0.f;
  for (int64_t i = tid; i < na4; i += nth) {
    const float4 x = a[i], y = b[i];
    acc += x.x + x.y + x.z + x.w + y.x + y.y + y.z + y.w;
  }
  for (int64_t i = tid; i < nc4; i += nth) {
    const float4 z = c[i];
    acc += z.x + z.y + z.z + z.w;
  }
  for (int64_t i = tid; i < no4; i += nth) {
    float4 v; v.x = acc; v.y = acc; v.z = acc; v.w = acc;
    o1[i] = v; o2[i] = v;
  }
  if (acc == 12345.f) sink[0] = acc;
}

extern "C" int exp_stream_launch(const void* a, const void* b, const void* c, int64_t na4, int64_t nc4,
                                 void* o1, void* o2, int64_t no4, void* sink, int grid, void* st) {
  hipLaunchKernelGGL(exp_stream, dim3(grid), dim3(256), 0, (hipStream_t)st, (const float4*)a,
                     (const float4*)b, (const float4*)c, na4, nc4, (float4*)o1, (float4*)o2, no4,
                     (float*)sink);
  return (int)hipGetLastError();
}
