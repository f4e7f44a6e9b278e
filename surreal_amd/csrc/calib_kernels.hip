// calib_kernels.hip — measurement only (not part of the reference API): the
// fixed-work calibration launches bench.py runs right before its timed region
// and the clock probe that runs beside it, so a bench line carries what the box
// delivered that day (MI355X_MICROARCH.md "DVFS give-back": one binary differs
// by up to ~12 % across MI355X devices) next to the learner's own number.
//
//   calib_mfma_kernel    v_mfma_f32_32x32x2_f32 chains on register operands
//                        (random data: zero operands clock higher), 4
//                        independent accumulators per wave, 2 waves per SIMD;
//                        4096 flops per MFMA; per-workgroup clock stamps.
//   calib_stream_kernel  y = x * s as float4, resident grid-stride: 8 bytes per
//                        element over a working set the caller sizes > MALL.
//   clock_probe_kernel   one wave that sleeps in a loop until a stop flag (set
//                        by clock_probe_stop_kernel on another stream) or its
//                        realtime budget runs out, then stores its s_memtime /
//                        s_memrealtime deltas: the average shader clock over
//                        the window = d(memtime) / d(memrealtime) x 100 MHz.
// Stamps go to a buffer of their own (vector stores), never into an output.
#include <hip/hip_runtime.h>
#include "smi_internal.hpp"

namespace smi {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4c __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return x;
}
__device__ __forceinline__ float rnd(uint32_t s) {
  return (float)(hash32(s) >> 8) * (1.0f / 16777216.0f) - 0.5f;
}

__global__ void __launch_bounds__(256, 2)
calib_mfma_kernel(int iters, float* __restrict__ out, long long* __restrict__ stamps) {
  const uint32_t g = blockIdx.x * 256u + threadIdx.x;
  float a0 = rnd(4 * g), a1 = rnd(4 * g + 1), b0 = rnd(4 * g + 2), b1 = rnd(4 * g + 3);
  f32x16 c0, c1, c2, c3;
#pragma unroll
  for (int i = 0; i < 16; ++i) { c0[i] = 0.f; c1[i] = 0.f; c2[i] = 0.f; c3[i] = 0.f; }
  const long long m0 = __builtin_amdgcn_s_memtime();
  const long long r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < iters; ++it) {
    c0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, c3, 0, 0, 0);
  }
  const long long m1 = __builtin_amdgcn_s_memtime();
  const long long r1 = __builtin_amdgcn_s_memrealtime();
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) s += c0[i] + c1[i] + c2[i] + c3[i];
  out[g] = s;
  if (threadIdx.x == 0) {
    stamps[2 * blockIdx.x] = m1 - m0;
    stamps[2 * blockIdx.x + 1] = r1 - r0;
  }
}

__global__ void __launch_bounds__(256)
calib_stream_kernel(const f32x4c* __restrict__ x, f32x4c* __restrict__ y, int64_t n4, float s) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += stride) {
    f32x4c v = __builtin_nontemporal_load(x + i);
    __builtin_nontemporal_store(v * s, y + i);
  }
}

__global__ void __launch_bounds__(64)
clock_probe_kernel(const int* __restrict__ flag, long long max_ticks, long long* __restrict__ out) {
  const long long m0 = __builtin_amdgcn_s_memtime();
  const long long r0 = __builtin_amdgcn_s_memrealtime();
  long long r = r0;
  // every wave leaves: on the flag, or when max_ticks of the 100 MHz counter pass
  while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0 &&
         r - r0 < max_ticks) {
    __builtin_amdgcn_s_sleep(64);
    r = __builtin_amdgcn_s_memrealtime();
  }
  const long long m1 = __builtin_amdgcn_s_memtime();
  r = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) {
    out[0] = m1 - m0;
    out[1] = r - r0;
    out[2] = r - r0 >= max_ticks;       // 1 = timed out (the window is not the caller's)
  }
}

__global__ void clock_probe_stop_kernel(int* __restrict__ flag, int v) {
  if (threadIdx.x == 0) __hip_atomic_store(flag, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace smi

using namespace smi;

extern "C" {

int smi_calib_mfma(int n_wg, int iters, float* out, long long* stamps, void* stream) {
  if (n_wg <= 0 || iters <= 0 || !out || !stamps)
    return set_error(SMI_E_ARG, "calib_mfma: n_wg, iters > 0 and out[n_wg * 256], stamps[2 n_wg]");
  hipLaunchKernelGGL(calib_mfma_kernel, dim3(n_wg), dim3(256), 0, static_cast<hipStream_t>(stream),
                     iters, out, stamps);
  return check_launch("calib_mfma_kernel");
}

int smi_calib_stream(const float* x, float* y, int64_t n, void* stream) {
  if (!x || !y || n <= 0 || n % 4 || (reinterpret_cast<uintptr_t>(x) & 15) ||
      (reinterpret_cast<uintptr_t>(y) & 15))
    return set_error(SMI_E_ARG, "calib_stream: 16-byte aligned x, y and n a positive multiple of 4");
  const int grid = resident_grid(calib_stream_kernel, 256, 0);
  hipLaunchKernelGGL(calib_stream_kernel, dim3(grid), dim3(256), 0, static_cast<hipStream_t>(stream),
                     reinterpret_cast<const f32x4c*>(x), reinterpret_cast<f32x4c*>(y), n / 4,
                     1.0000001f);
  return check_launch("calib_stream_kernel");
}

int smi_clock_probe(const int* flag, long long max_ticks, long long* out3, void* stream) {
  if (!flag || !out3 || max_ticks <= 0 || max_ticks > 3000000000LL)
    return set_error(SMI_E_ARG, "clock_probe: flag, out3 and 0 < max_ticks <= 30 s of 100 MHz ticks");
  hipLaunchKernelGGL(clock_probe_kernel, dim3(1), dim3(64), 0, static_cast<hipStream_t>(stream),
                     flag, max_ticks, out3);
  return check_launch("clock_probe_kernel");
}

int smi_clock_probe_stop(int* flag, int value, void* stream) {
  if (!flag) return set_error(SMI_E_ARG, "clock_probe_stop: flag");
  hipLaunchKernelGGL(clock_probe_stop_kernel, dim3(1), dim3(64), 0,
                     static_cast<hipStream_t>(stream), flag, value);
  return check_launch("clock_probe_stop_kernel");
}

}  // extern "C"
