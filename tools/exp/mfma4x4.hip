// Layout + issue-rate probe of v_mfma_f32_4x4x1_16b_f32 with A broadcast from
// block 0 (cbsz 4, abid 0): expected D[lane][i] = A(lane i of block 0) * B(lane).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void layout_kernel(float* out) {
  const int l = threadIdx.x;
  const float a = 100.f + l, b = 1.f + l;
  f32x4 c = {0.f, 0.f, 0.f, 0.f};
  c = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c, 4, 0, 0);
  for (int i = 0; i < 4; ++i) out[l * 4 + i] = c[i];
}

template <int CH>
__global__ void rate_kernel(float* out, long long* cyc, int n) {
  const int l = threadIdx.x & 63;
  float a = 1e-3f * l, b = 1e-3f * (l + 1);
  f32x4 c[CH];
  for (int j = 0; j < CH; ++j) c[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  __syncthreads();
  const long long t0 = clock64();
  for (int i = 0; i < n; ++i) {
#pragma unroll
    for (int j = 0; j < CH; ++j) c[j] = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c[j], 4, 0, 0);
  }
  const long long t1 = clock64();
  float s = 0.f;
  for (int j = 0; j < CH; ++j) s += c[j][0] + c[j][1] + c[j][2] + c[j][3];
  out[threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

int main() {
  float* d; long long* cy;
  hipMalloc(&d, 4096 * 4); hipMalloc(&cy, 8);
  layout_kernel<<<1, 64>>>(d);
  float h[256];
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  int bad = 0;
  for (int l = 0; l < 64; ++l)
    for (int i = 0; i < 4; ++i) {
      const float e = (100.f + i) * (1.f + l);
      if (h[l * 4 + i] != e) { if (bad < 8) printf("lane %d reg %d got %g want %g\n", l, i, h[l * 4 + i], e); ++bad; }
    }
  printf("layout mismatches: %d\n", bad);
  const int n = 4096;
  long long c;
  rate_kernel<1><<<1, 64>>>(d, cy, n); hipMemcpy(&c, cy, 8, hipMemcpyDeviceToHost);
  printf("1 chain: %.2f cycles/mfma\n", (double)c / n);
  rate_kernel<2><<<1, 64>>>(d, cy, n); hipMemcpy(&c, cy, 8, hipMemcpyDeviceToHost);
  printf("2 chains: %.2f cycles/mfma\n", (double)c / (2.0 * n));
  rate_kernel<4><<<1, 64>>>(d, cy, n); hipMemcpy(&c, cy, 8, hipMemcpyDeviceToHost);
  printf("4 chains: %.2f cycles/mfma\n", (double)c / (4.0 * n));
  rate_kernel<4><<<1, 256>>>(d, cy, n); hipMemcpy(&c, cy, 8, hipMemcpyDeviceToHost);
  printf("4 chains, 4 waves: %.2f cycles/mfma (wave 0)\n", (double)c / (4.0 * n));
  rate_kernel<4><<<1, 512>>>(d, cy, n); hipMemcpy(&c, cy, 8, hipMemcpyDeviceToHost);
  printf("4 chains, 8 waves: %.2f cycles/mfma (wave 0)\n", (double)c / (4.0 * n));
  return 0;
}
