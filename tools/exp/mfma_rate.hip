// f32 MFMA rate calibration for the grouped dW launch (diagnostic only, not
// product code).  Each wave runs the dW kernel's inner step: a 64 x 64 output
// tile as 4 x 4 v_mfma_f32_16x16x4_f32 accumulators, per 4-row step one
// 16-byte operand load of each matrix (dY rows, X rows), DWD_P = 4 steps in
// flight.  MODE 0 = the MFMAs alone (operands from registers), MODE 1 = with
// the operand stream over a C3-sized pair of row-major matrices (21504 rows x
// 400 | 144 floats), the workgroups dealt to (m-tile, n-tile, row slab) as the
// grouped launch does.  Prints the algorithmic TF/s and the in-kernel clock
// (clock64 delta over the 100 MHz wall-clock delta, median over workgroups).
//   hipcc -O3 --offload-arch=gfx950 tools/exp/mfma_rate.hip -o /tmp/mfma_rate
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int R = 21504, MA = 400, NB = 144, P = 4, RS = 16;

template <int MODE, int OCC>
__global__ void __launch_bounds__(256, OCC)
rate_kernel(const float* __restrict__ A, const float* __restrict__ B, int kc, int reps,
            float* out, unsigned long long* clk) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, li = lane & 15, lk = lane >> 4;
  const int w = blockIdx.x;
  const int mt = w % 7, nt = (w / 7) % 3, slab = (w / 21) % (R / kc);
  const int m0 = std::min(64 * mt, MA - 64), n0 = std::min(64 * nt, NB - 64);
  f32x4 acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  const unsigned long long c0 = clock64(), t0 = wall_clock64();
  const int nsteps = kc / RS;
  for (int rep = 0; rep < reps; ++rep) {
    const int rw = slab * kc + 4 * wave + lk;
    const float* pa = A + (int64_t)rw * MA + m0 + 4 * li;
    const float* pb = B + (int64_t)rw * NB + n0 + 4 * li;
    // global loads spelled out, prologue pinned in step order, refills
    // unconditional (the buffers carry P * RS rows of padding): the product
    // dW loop's schedule (vmcnt(6) before each step)
    using gv4 = const __attribute__((address_space(1))) f32x4;
    f32x4 av[P], bv[P];
#pragma unroll
    for (int p = 0; p < P; ++p) {
      av[p] = *(gv4*)pa; pa += RS * MA;
      bv[p] = *(gv4*)pb; pb += RS * NB;
      __builtin_amdgcn_sched_barrier(0);
    }
    for (int s0 = 0; s0 < nsteps; s0 += P) {
#pragma unroll
      for (int p = 0; p < P; ++p) {
#pragma unroll
        for (int b = 0; b < 4; ++b)
#pragma unroll
          for (int a = 0; a < 4; ++a)
            acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[p][a], bv[p][b], acc[a][b], 0, 0, 0);
        if (MODE == 1) {
          av[p] = *(gv4*)pa; pa += RS * MA;
          bv[p] = *(gv4*)pb; pb += RS * NB;
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  }
  const unsigned long long c1 = clock64(), t1 = wall_clock64();
  float s = 0.f;
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) s += acc[a][b][0] + acc[a][b][1] + acc[a][b][2] + acc[a][b][3];
  out[(int64_t)blockIdx.x * 256 + threadIdx.x] = s;
  if (threadIdx.x == 0) { clk[2 * blockIdx.x] = c1 - c0; clk[2 * blockIdx.x + 1] = t1 - t0; }
}

template <int MODE, int OCC>
static void run(const float* A, const float* B, float* out, unsigned long long* clk, int kc, int reps) {
  const int nwg = 256 * OCC;
  auto launch = [&] { hipLaunchKernelGGL((rate_kernel<MODE, OCC>), dim3(nwg), dim3(256), 0, 0, A, B, kc, reps, out, clk); };
  for (int i = 0; i < 200; ++i) launch();                      // >= ~1 s of warm load
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  std::vector<float> ts;
  for (int i = 0; i < 21; ++i) {
    CK(hipEventRecord(e0)); launch(); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ts.push_back(ms);
  }
  std::sort(ts.begin(), ts.end());
  const double ms = ts[ts.size() / 2];
  std::vector<unsigned long long> h(2 * nwg);
  CK(hipMemcpy(h.data(), clk, h.size() * 8, hipMemcpyDeviceToHost));
  std::vector<double> ghz;
  for (int i = 0; i < nwg; ++i) if (h[2 * i + 1]) ghz.push_back((double)h[2 * i] / (double)h[2 * i + 1] * 0.1);
  std::sort(ghz.begin(), ghz.end());
  const double flop = (double)nwg * 4 * reps * (kc / RS) * 16 * 2048.0;
  printf("{\"mode\": %d, \"wg_per_cu\": %d, \"kc\": %d, \"ms\": %.4f, \"tflops\": %.1f, \"frac_157\": %.3f, \"clock_ghz_med\": %.3f}\n",
         MODE, OCC, kc, ms, flop / ms / 1e9, flop / ms / 1e9 / 157.3, ghz[ghz.size() / 2]);
  fflush(stdout);
}

int main() {
  float *A, *B, *out;
  unsigned long long* clk;
  CK(hipMalloc(&A, (size_t)(R + P * RS) * MA * 4)); CK(hipMalloc(&B, (size_t)(R + P * RS) * NB * 4));
  CK(hipMalloc(&out, (size_t)1024 * 256 * 4)); CK(hipMalloc(&clk, (size_t)2048 * 8));
  {
    std::vector<float> h((size_t)R * MA);
    unsigned s = 12345u;
    for (auto& v : h) { s = s * 1664525u + 1013904223u; v = (float)((s >> 9) & 0xffff) / 65536.f - 0.5f; }
    CK(hipMemcpy(A, h.data(), (size_t)R * MA * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(B, h.data(), (size_t)R * NB * 4, hipMemcpyHostToDevice));
  }
  // 576-row slabs (36 per tile) as at C3; reps stretch a launch to ~1 ms
  if (getenv("RATE_SMALL")) {      // a rank's share (3200 rows): 448-row slabs, one pass
    run<0, 1>(A, B, out, clk, 448, 1); run<1, 1>(A, B, out, clk, 448, 1);
    run<0, 2>(A, B, out, clk, 448, 1); run<1, 2>(A, B, out, clk, 448, 1);
    run<1, 1>(A, B, out, clk, 1344, 1); run<1, 1>(A, B, out, clk, 448, 20);
    return 0;
  }
  run<1, 2>(A, B, out, clk, 576, 20); run<1, 3>(A, B, out, clk, 576, 14);
  run<0, 3>(A, B, out, clk, 576, 1);  // one pass, the dW launch's size
  run<1, 3>(A, B, out, clk, 576, 1);
  run<0, 3>(A, B, out, clk, 1344, 1); // the C3 launch's rows per workgroup
  run<1, 3>(A, B, out, clk, 1344, 1);
  return 0;
}
