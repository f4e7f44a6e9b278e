// Round 6: the VALU LSTM forward's W_hh prologue at a rank's batch (diagnostic
// only, not product code).  128 workgroups x 448 threads each load one LSTM's
// W_hh [400][100] into registers the way lstm_fwd_q_kernel<28, ., ., 2> does
// (thread (u, q) = gate rows j*H + u over k runs 16 i + 4 q .. + 3: per load
// instruction a wave touches 16 rows x 64 B) -- LAYOUT 0 -- or from a copy
// swizzled to the register order (slot s = j*7 + i, thread t: [s][448] float4,
// a wave's load instruction = 1 KB contiguous) -- LAYOUT 1.  Each is timed
// (HIP events around that launch alone) with the weights untouched since the
// previous launch (clean) and right after a kernel that rewrote them as Adam
// does (dirty: read-modify-write of every element on one XCD's workgroups).
//   hipcc -O3 --offload-arch=gfx950 tools/exp/lstm_prologue.hip -o tools/exp/lstm_prologue
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int H = 100, G4 = 400, NT = 448, NS = 28;

template <int LAYOUT>
__global__ void __launch_bounds__(NT) load_kernel(const float* __restrict__ w, float* __restrict__ out) {
  const int tid = threadIdx.x, u = tid >> 2, q = tid & 3;
  const int uc = u < H ? u : H - 1;
  float4 v[NS];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < 7; ++i) {
      if (LAYOUT == 0) {
        const int k = 16 * i + 4 * q;
        v[j * 7 + i] = k + 3 < H ? *reinterpret_cast<const float4*>(w + (int64_t)(j * H + uc) * H + k)
                                 : float4{0.f, 0.f, 0.f, 0.f};
      } else {
        v[j * 7 + i] = reinterpret_cast<const float4*>(w)[(j * 7 + i) * NT + tid];
      }
    }
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < NS; ++k) s += (v[k].x + v[k].y) + (v[k].z + v[k].w);
  out[(int64_t)blockIdx.x * NT + tid] = s;
}

// Adam-like rewrite of n floats: p = p * (1 - 1e-7) + 1e-9 (grid-stride)
__global__ void __launch_bounds__(256) dirty_kernel(float* __restrict__ p, int n) {
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) p[i] = p[i] * 0.9999999f + 1e-9f;
}

template <int LAYOUT>
static float run(const float* w, float* wmut, int nw, float* out, bool dirty, int iters) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<float> ts;
  for (int it = 0; it < iters + 3; ++it) {
    if (dirty) hipLaunchKernelGGL(dirty_kernel, dim3(64), dim3(256), 0, 0, wmut, nw);
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(load_kernel<LAYOUT>, dim3(128), dim3(NT), 0, 0, w, out);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (it >= 3) ts.push_back(ms * 1e3f);
  }
  std::sort(ts.begin(), ts.end());
  return ts[ts.size() / 2];
}

__global__ void empty_kernel() {}

int main() {
  std::vector<float> hw((size_t)G4 * H), hs((size_t)NS * NT * 4, 0.f);
  srand(1);
  for (auto& v : hw) v = (float)rand() / RAND_MAX - 0.5f;
  for (int t = 0; t < NT; ++t) {
    const int u = t >> 2, q = t & 3, uc = u < H ? u : H - 1;
    for (int j = 0; j < 4; ++j)
      for (int i = 0; i < 7; ++i)
        for (int c = 0; c < 4; ++c) {
          const int k = 16 * i + 4 * q + c;
          hs[((size_t)(j * 7 + i) * NT + t) * 4 + c] = k < H && 16 * i + 4 * q + 3 < H ? hw[(size_t)(j * H + uc) * H + k] : 0.f;
        }
  }
  float *dw, *ds, *out;
  CK(hipMalloc(&dw, hw.size() * 4));
  CK(hipMalloc(&ds, hs.size() * 4));
  CK(hipMalloc(&out, (size_t)128 * NT * 4));
  CK(hipMemcpy(dw, hw.data(), hw.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(ds, hs.data(), hs.size() * 4, hipMemcpyHostToDevice));
  // launch overhead of an event-bracketed empty launch
  {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<float> ts;
    for (int it = 0; it < 33; ++it) {
      CK(hipEventRecord(e0));
      hipLaunchKernelGGL(empty_kernel, dim3(128), dim3(NT), 0, 0);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (it >= 3) ts.push_back(ms * 1e3f);
    }
    std::sort(ts.begin(), ts.end());
    printf("{\"empty_launch_us\": %.2f}\n", ts[ts.size() / 2]);
  }
  printf("{\"layout\": \"rows (product)\", \"clean_us\": %.2f, \"dirty_us\": %.2f}\n",
         run<0>(dw, dw, (int)hw.size(), out, false, 30), run<0>(dw, dw, (int)hw.size(), out, true, 30));
  printf("{\"layout\": \"swizzled\", \"clean_us\": %.2f, \"dirty_us\": %.2f}\n",
         run<1>(ds, ds, (int)hs.size(), out, false, 30), run<1>(ds, ds, (int)hs.size(), out, true, 30));
  return 0;
}
