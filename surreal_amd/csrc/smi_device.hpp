// smi_device.hpp — CDNA4 (gfx950) device building blocks for the SURREAL learner
// hot path: LDS-resident 64-row tiles, fp32 MFMA (v_mfma_f32_16x16x4_f32) dense
// layers with fused bias/activation epilogues and their backward passes, and
// wave/block reductions.  Every helper is templated on the workgroup size NT
// (a multiple of 64); the fused epoch kernels run 512 threads (8 waves = 2 per
// SIMD), the streaming kernels 256.
//
// MFMA operand maps (16x16x4 f32, cdna_hip_programming.md §3):
//   A[i = lane&15][k = lane>>4], B[k = lane>>4][j = lane&15],
//   D[row = (lane>>4)*4 + reg][col = lane&15].
// The f32 MFMA is an exact k-ordered fmaf chain, so these layers are fp32
// exact up to summation order (parity bar: 1e-5 relative vs the CPU oracle).
//
// Latency: at learner sizes every dense layer is a chain of dependent
// LDS-read -> MFMA steps, so the k-loops load 8 k-steps of both operands into
// registers before issuing the 8 MFMAs (one LDS round trip per 8 MFMAs).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace smi {

constexpr int kWG = 256;          // default threads per workgroup
constexpr int kNW = kWG / 64;     // waves of a default workgroup
constexpr int kRT = 64;           // rows per tile
constexpr int kMaxW = 16;         // max waves per workgroup (scratch sizing)

typedef float f32x4 __attribute__((ext_vector_type(4)));

enum { ACT_NONE = 0, ACT_RELU = 1, ACT_TANH = 2 };

// LDS leading dimension for a K-wide row: >= roundup(K,4) and == 2 (mod 32), so
// the A-operand column reads of a 32-lane half (16 rows at k, 16 rows at k+1)
// land on 32 distinct banks.
__host__ __device__ inline int pad_ld(int k) {
  const int k4 = (k + 3) & ~3;
  const int r = (k4 - 2) & 31;
  return k4 + (32 - r);
}
__host__ __device__ inline int round4(int k) { return (k + 3) & ~3; }
// Leading dim of narrow (<= ~16 column) output/gradient tiles: odd stride, a few
// 2-way conflicts at most, and 3-7x less LDS than pad_ld for 1..8 columns.
__host__ __device__ inline int pad_small(int k) { return round4(k) + 1; }

template <int ACT>
__device__ __forceinline__ float act_f(float x) {
  if constexpr (ACT == ACT_RELU) return x > 0.f ? x : 0.f;
  else if constexpr (ACT == ACT_TANH) return tanhf(x);
  else return x;
}

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// ---------------------------------------------------------------- reductions
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
// Block-wide sum; `scratch` is >= NT/64 doubles of LDS.  Every thread gets the
// result.  Fixed order (deterministic).
template <int NT = kWG>
__device__ __forceinline__ double block_sum_d(double v, double* scratch) {
  v = wave_sum_d(v);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) scratch[wave] = v;
  __syncthreads();
  double s = 0.0;
#pragma unroll
  for (int w = 0; w < NT / 64; ++w) s += scratch[w];
  __syncthreads();
  return s;
}
template <int NT = kWG>
__device__ __forceinline__ float block_sum_f(float v, double* scratch) {
  return (float)block_sum_d<NT>((double)v, scratch);
}

// --------------------------------------------------------------- dense layers
// SMI_DENSE_NOINLINE (developer variant) emits each dense helper once instead of
// inlining it at every call site: smaller code, at the price of call overhead.
#ifdef SMI_DENSE_NOINLINE
#define SMI_DENSE __device__ __attribute__((noinline))
#else
#define SMI_DENSE __device__
#endif
// Forward: Y[r][n] = act(b[n] + sum_k X[r][k] * W[n][k]),  r in [0,64), n in [0,N)
//   X: LDS [64][ldx], columns [K, round4(K)) must be zero (finite).
//   W: [N][ldw] row-major (k contiguous) in LDS or global; b: [N].
//   Y: LDS [64][ldy]; only columns < N are written.
// 16x16 output tiles are dealt round-robin to the NT/64 waves.
template <int ACT, int NT = kWG>
SMI_DENSE void dense_fwd(const float* __restrict__ X, int ldx,
                          const float* __restrict__ W, int ldw,
                          const float* __restrict__ b, int K, int N,
                          float* __restrict__ Y, int ldy) {
  constexpr int NW = NT / 64;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int li = lane & 15, lk = lane >> 4;
  const int CT = (N + 15) >> 4;
  const int K4 = round4(K);
  for (int t = wave; t < 4 * CT; t += NW) {
    const int rb = t & 3, ct = t >> 2;
    const int n = ct * 16 + li;
    const bool nv = n < N;
    const float* xp = X + (rb * 16 + li) * ldx + lk;
    const float* wp = W + (nv ? n : 0) * ldw + lk;
    const float bn = nv ? b[n] : 0.f;
    f32x4 acc = {bn, bn, bn, bn};
    int k0 = 0;
    for (; k0 + 32 <= K4; k0 += 32) {
      float a[8], w[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        a[u] = xp[k0 + 4 * u];
        w[u] = (nv && (k0 + 4 * u + lk) < K) ? wp[k0 + 4 * u] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) acc = mfma4(a[u], w[u], acc);
    }
    for (; k0 < K4; k0 += 4) {
      const float a = xp[k0];
      const float w = (nv && (k0 + lk) < K) ? wp[k0] : 0.f;
      acc = mfma4(a, w, acc);
    }
    if (nv) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        Y[(rb * 16 + lk * 4 + i) * ldy + n] = act_f<ACT>(acc[i]);
    }
  }
}

// Backward to the layer input: dX[r][k] = mask(Xact[r][k]) * sum_n G[r][n] W[n][k]
//   PREV_ACT = activation that produced X (ACT_RELU: mask Xact > 0; ACT_NONE: none)
//   G: LDS [64][ldg], columns [N, round4(N)) finite.  dX must not alias G.
template <int PREV_ACT, int NT = kWG>
SMI_DENSE void dense_bwd_dx(const float* __restrict__ G, int ldg,
                             const float* __restrict__ W, int ldw, int K, int N,
                             const float* __restrict__ Xact, int ldx,
                             float* __restrict__ dX, int lddx) {
  constexpr int NW = NT / 64;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int li = lane & 15, lk = lane >> 4;
  const int CT = (K + 15) >> 4;
  const int N4 = round4(N);
  for (int t = wave; t < 4 * CT; t += NW) {
    const int rb = t & 3, ct = t >> 2;
    const int k = ct * 16 + li;
    const bool kv = k < K;
    const float* gp = G + (rb * 16 + li) * ldg + lk;
    const float* wp = W + lk * ldw + (kv ? k : 0);
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    int n0 = 0;
    for (; n0 + 32 <= N4; n0 += 32) {
      float a[8], w[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        a[u] = gp[n0 + 4 * u];
        w[u] = (kv && (n0 + 4 * u + lk) < N) ? wp[(n0 + 4 * u) * ldw] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) acc = mfma4(a[u], w[u], acc);
    }
    for (; n0 < N4; n0 += 4) {
      const float a = gp[n0];
      const float w = (kv && (n0 + lk) < N) ? wp[n0 * ldw] : 0.f;
      acc = mfma4(a, w, acc);
    }
    if (kv) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = rb * 16 + lk * 4 + i;
        float v = acc[i];
        if constexpr (PREV_ACT == ACT_RELU) v = Xact[r * ldx + k] > 0.f ? v : 0.f;
        dX[r * lddx + k] = v;
      }
    }
  }
}

// Weight/bias gradients, accumulated: gW[n][k] += sum_r G[r][n] X[r][k],
// gb[n] += sum_r G[r][n], over the 64 rows of the tile (rows that are not
// valid must carry G == 0 and finite X).
template <int NT = kWG>
SMI_DENSE void dense_bwd_dw(const float* __restrict__ G, int ldg,
                             const float* __restrict__ X, int ldx, int K, int N,
                             float* __restrict__ gW, int ldgw,
                             float* __restrict__ gb) {
  constexpr int NW = NT / 64;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int li = lane & 15, lk = lane >> 4;
  const int NTL = (N + 15) >> 4, KT = (K + 15) >> 4;
  for (int t = wave; t < NTL * KT; t += NW) {
    const int nt = t / KT, kt = t - nt * KT;
    const int na = nt * 16 + li;   // A-operand row (output n)
    const int kb = kt * 16 + li;   // B-operand col (input k)
    const bool nav = na < N, kbv = kb < K;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int h = 0; h < kRT / 32; ++h) {
      float a[8], x[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int r = h * 32 + 4 * u + lk;
        a[u] = nav ? G[r * ldg + na] : 0.f;
        x[u] = kbv ? X[r * ldx + kb] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) acc = mfma4(a[u], x[u], acc);
    }
    if (kbv) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int nn = nt * 16 + lk * 4 + i;
        if (nn < N) gW[nn * ldgw + kb] += acc[i];
      }
    }
  }
  for (int n = threadIdx.x; n < N; n += NT) {
    float s = 0.f;
#pragma unroll 8
    for (int r = 0; r < kRT; ++r) s += G[r * ldg + n];
    gb[n] += s;
  }
}

// ------------------------------------------------------------ MLP layouts
// Flat (global, torch) layout and padded (LDS) layout of a 3-layer MLP
// in -> h1 -> h2 -> out [+ log_var(out)].
struct MlpLayout {
  int in, h1, h2, out, lv;
  // flat offsets
  int fW1, fb1, fW2, fb2, fW3, fb3, flv, fcount;
  // padded LDS offsets and leading dims
  int ld1, ld2, ld3;
  int pW1, pb1, pW2, pb2, pW3, pb3, plv, pcount;
};

__host__ __device__ inline MlpLayout mlp_layout(int in, int h1, int h2, int out, int lv) {
  MlpLayout L;
  L.in = in; L.h1 = h1; L.h2 = h2; L.out = out; L.lv = lv;
  L.fW1 = 0;
  L.fb1 = L.fW1 + h1 * in;
  L.fW2 = L.fb1 + h1;
  L.fb2 = L.fW2 + h2 * h1;
  L.fW3 = L.fb2 + h2;
  L.fb3 = L.fW3 + out * h2;
  L.flv = L.fb3 + out;
  L.fcount = L.flv + (lv ? out : 0);
  L.ld1 = pad_ld(in); L.ld2 = pad_ld(h1); L.ld3 = pad_ld(h2);
  L.pW1 = 0;
  L.pb1 = L.pW1 + h1 * L.ld1;
  L.pW2 = round4(L.pb1 + h1);
  L.pb2 = L.pW2 + h2 * L.ld2;
  L.pW3 = round4(L.pb2 + h2);
  L.pb3 = L.pW3 + out * L.ld3;
  L.plv = round4(L.pb3 + out);
  L.pcount = round4(L.plv + (lv ? out : 0));
  return L;
}

// flat index -> padded index
__device__ inline int mlp_flat_to_pad(const MlpLayout& L, int i) {
  if (i < L.fb1) { const int n = i / L.in; return L.pW1 + n * L.ld1 + (i - n * L.in); }
  if (i < L.fW2) return L.pb1 + (i - L.fb1);
  if (i < L.fb2) { const int j = i - L.fW2; const int n = j / L.h1; return L.pW2 + n * L.ld2 + (j - n * L.h1); }
  if (i < L.fW3) return L.pb2 + (i - L.fb2);
  if (i < L.fb3) { const int j = i - L.fW3; const int n = j / L.h2; return L.pW3 + n * L.ld3 + (j - n * L.h2); }
  if (i < L.flv) return L.pb3 + (i - L.fb3);
  return L.plv + (i - L.flv);
}

// Pointer view of an MLP parameter set, either the padded LDS image or the flat
// global buffer (leading dims = true widths).
struct MlpView {
  const float *W1, *b1, *W2, *b2, *W3, *b3, *lv;
  int ld1, ld2, ld3;
};
__device__ inline MlpView view_padded(const MlpLayout& L, const float* P) {
  MlpView v;
  v.W1 = P + L.pW1; v.b1 = P + L.pb1; v.W2 = P + L.pW2; v.b2 = P + L.pb2;
  v.W3 = P + L.pW3; v.b3 = P + L.pb3; v.lv = P + L.plv;
  v.ld1 = L.ld1; v.ld2 = L.ld2; v.ld3 = L.ld3;
  return v;
}
__device__ inline MlpView view_flat(const MlpLayout& L, const float* F) {
  MlpView v;
  v.W1 = F + L.fW1; v.b1 = F + L.fb1; v.W2 = F + L.fW2; v.b2 = F + L.fb2;
  v.W3 = F + L.fW3; v.b3 = F + L.fb3; v.lv = F + L.flv;
  v.ld1 = L.in; v.ld2 = L.h1; v.ld3 = L.h2;
  return v;
}

// Load a flat MLP buffer into LDS (padded); the padding is zeroed.  The global
// loads of a thread are issued 8 at a time before their LDS stores.
template <int NT = kWG>
__device__ inline void mlp_load_lds(const MlpLayout& L, const float* __restrict__ flat,
                                    float* __restrict__ P) {
  for (int i = threadIdx.x; i < L.pcount; i += NT) P[i] = 0.f;
  __syncthreads();
  for (int base = 0; base < L.fcount; base += 8 * NT) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int i = base + u * NT + threadIdx.x;
      v[u] = i < L.fcount ? flat[i] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int i = base + u * NT + threadIdx.x;
      if (i < L.fcount) P[mlp_flat_to_pad(L, i)] = v[u];
    }
  }
  __syncthreads();
}
template <int NT = kWG>
__device__ inline void mlp_store_flat(const MlpLayout& L, const float* __restrict__ P,
                                      float* __restrict__ flat) {
  for (int i = threadIdx.x; i < L.fcount; i += NT) flat[i] = P[mlp_flat_to_pad(L, i)];
}

// Load a 64-row observation tile into LDS X[64][ldx] (row r = tile row), with
// the ZFilter of z_filter.py:59-79 applied when zmean != nullptr.  Rows >= nrows
// and columns >= dim are zero.
template <int NT = kWG>
__device__ inline void load_obs_tile(const float* __restrict__ src, int64_t row_stride,
                                     int nrows, int dim, const float* zmean,
                                     const float* zstd, float* __restrict__ X, int ldx) {
  const int total = kRT * ldx;
  for (int e = threadIdx.x; e < total; e += NT) {
    const int r = e / ldx, c = e - r * ldx;
    float v = 0.f;
    if (r < nrows && c < dim) {
      v = src[(int64_t)r * row_stride + c];
      if (zmean) {
        v = (v - zmean[c]) / zstd[c];
        v = fminf(fmaxf(v, -5.f), 5.f);
      }
    }
    X[e] = v;
  }
}

// ZFilter running mean / std per column (z_filter.py:69-72):
//   mean = sum / count; std = max(sqrt(sumsq/count - mean^2), eps)
template <int NT = kWG>
__device__ inline void zfilter_colstats(const float* sum, const float* sumsq,
                                        const float* count, float eps, int dim,
                                        float* zmean, float* zstd) {
  const float cnt = count[0];
  for (int c = threadIdx.x; c < dim; c += NT) {
    const float mean = sum[c] / cnt;
    const float sq = sumsq[c] / cnt;
    const float var = sq - mean * mean;
    float sd = sqrtf(var);
    sd = (sd < eps) ? eps : sd;   // torch.clamp(min=eps); NaN stays NaN
    zmean[c] = mean;
    zstd[c] = sd;
  }
}

}  // namespace smi
