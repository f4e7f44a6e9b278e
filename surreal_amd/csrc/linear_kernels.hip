// linear_kernels.hip — layer-by-layer fp32 MFMA GEMMs for networks whose
// parameters do not fit one CU's LDS (DDPG actor 300x200 / critic 400x300,
// builders.py:35-84; PPO heads 300x200).  Activations live in HBM (L2-resident
// at learner batch sizes); every dense layer's forward, input-gradient and
// weight-gradient are the same LDS-tiled GEMM with a different operand view
// and epilogue:
//   fwd:  Y[m][n]  = act(b[n] + sum_k X[m][k] W[n][k])
//   dX:   dX[m][k] = mask(Xact[m][k] > 0) * sum_n dY[m][n] W[n][k]
//   dW:   dW[n][k] (+)= sum_m dY[m][n] X[m][k]       (reduction over rows;
//         one workgroup owns an output tile: deterministic, no atomics)
// Tiles 64x64, K-steps of 16 staged through LDS, 4 waves x (16 rows x 64 cols)
// with v_mfma_f32_16x16x4_f32.
#include "smi_device.hpp"
#include "smi_internal.hpp"

namespace smi {

enum { EPI_FWD = 0, EPI_DX = 1, EPI_DW = 2 };

struct GemmArgs {
  int M, N, K;
  // A(m,k) = A[m*a_rs + k*a_cs], B(k,n) = B[k*b_rs + n*b_cs]
  const float* A; int64_t a_rs, a_cs;
  const float* B; int64_t b_rs, b_cs;
  float* C; int64_t ldc;          // C[m*ldc + n]
  const float* bias;              // EPI_FWD
  int act;                        // EPI_FWD: ACT_*
  const float* mask; int64_t ldm; // EPI_DX: zero where mask[m*ldm+n] <= 0 (may be null)
  int accumulate;                 // EPI_DW: C += result
};

template <int EPI>
__global__ void __launch_bounds__(kWG)
gemm_kernel(GemmArgs g) {
  __shared__ float As[64][17];
  __shared__ float Bs[16][68];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, lk = lane >> 4;
  const int m0 = blockIdx.x * 64, n0 = blockIdx.y * 64;
  f32x4 acc[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) acc[c] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int k0 = 0; k0 < g.K; k0 += 16) {
#pragma unroll
    for (int e = tid; e < 64 * 16; e += kWG) {
      const int r = e >> 4, kk = e & 15;
      const int m = m0 + r, k = k0 + kk;
      As[r][kk] = (m < g.M && k < g.K) ? g.A[(int64_t)m * g.a_rs + (int64_t)k * g.a_cs] : 0.f;
    }
#pragma unroll
    for (int e = tid; e < 16 * 64; e += kWG) {
      const int kk = e >> 6, c = e & 63;
      const int k = k0 + kk, n = n0 + c;
      Bs[kk][c] = (k < g.K && n < g.N) ? g.B[(int64_t)k * g.b_rs + (int64_t)n * g.b_cs] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < 16; ks += 4) {
      const float a = As[wave * 16 + li][ks + lk];
#pragma unroll
      for (int c = 0; c < 4; ++c)
        acc[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, Bs[ks + lk][c * 16 + li], acc[c], 0, 0, 0);
    }
    __syncthreads();
  }
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int n = n0 + c * 16 + li;
    if (n >= g.N) continue;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = m0 + wave * 16 + lk * 4 + i;
      if (m >= g.M) continue;
      float v = acc[c][i];
      float* dst = g.C + (int64_t)m * g.ldc + n;
      if constexpr (EPI == EPI_FWD) {
        v += g.bias ? g.bias[n] : 0.f;
        if (g.act == ACT_RELU) v = v > 0.f ? v : 0.f;
        else if (g.act == ACT_TANH) v = tanhf(v);
        *dst = v;
      } else if constexpr (EPI == EPI_DX) {
        if (g.mask) v = g.mask[(int64_t)m * g.ldm + n] > 0.f ? v : 0.f;
        *dst = v;
      } else {
        *dst = g.accumulate ? *dst + v : v;
      }
    }
  }
}

// column sums over rows: out[n] (+)= sum_m X[m*ldx + n]   (bias gradients)
__global__ void __launch_bounds__(kWG)
colsum_kernel(const float* __restrict__ X, int M, int N, int64_t ldx, float* out, int accumulate) {
  __shared__ float s[kNW][64];
  const int n = blockIdx.x * 64 + (threadIdx.x & 63);
  const int rl = threadIdx.x >> 6;
  float a = 0.f;
  if (n < N)
    for (int m = rl; m < M; m += kNW) a += X[(int64_t)m * ldx + n];
  s[rl][threadIdx.x & 63] = a;
  __syncthreads();
  if (rl == 0 && n < N) {
    float t = 0.f;
    for (int w = 0; w < kNW; ++w) t += s[w][threadIdx.x];
    out[n] = accumulate ? out[n] + t : t;
  }
}

static int gemm_launch(int epi, const GemmArgs& g, hipStream_t st) {
  if (g.M <= 0 || g.N <= 0) return SMI_OK;
  const dim3 grid((g.M + 63) / 64, (g.N + 63) / 64);
  if (epi == EPI_FWD) hipLaunchKernelGGL(gemm_kernel<EPI_FWD>, grid, dim3(kWG), 0, st, g);
  else if (epi == EPI_DX) hipLaunchKernelGGL(gemm_kernel<EPI_DX>, grid, dim3(kWG), 0, st, g);
  else hipLaunchKernelGGL(gemm_kernel<EPI_DW>, grid, dim3(kWG), 0, st, g);
  return check_launch("gemm_kernel");
}

int launch_linear_fwd(const float* X, int64_t ldx, int M, int K, const float* W, int64_t ldw,
                      const float* b, int N, int act, float* Y, int64_t ldy, hipStream_t st) {
  GemmArgs g{};
  g.M = M; g.N = N; g.K = K;
  g.A = X; g.a_rs = ldx; g.a_cs = 1;
  g.B = W; g.b_rs = 1; g.b_cs = ldw;        // B(k,n) = W[n][k]
  g.C = Y; g.ldc = ldy; g.bias = b; g.act = act;
  return gemm_launch(EPI_FWD, g, st);
}

int launch_linear_bwd_dx(const float* dY, int64_t ldg, int M, int N, const float* W, int64_t ldw,
                         int K, const float* mask, int64_t ldm, float* dX, int64_t lddx,
                         hipStream_t st) {
  GemmArgs g{};
  g.M = M; g.N = K; g.K = N;
  g.A = dY; g.a_rs = ldg; g.a_cs = 1;
  g.B = W; g.b_rs = ldw; g.b_cs = 1;        // B(k=n', n=k') = W[n'][k']
  g.C = dX; g.ldc = lddx; g.mask = mask; g.ldm = ldm;
  return gemm_launch(EPI_DX, g, st);
}

int launch_linear_bwd_dw(const float* dY, int64_t ldg, int M, int N, const float* X, int64_t ldx,
                         int K, float* dW, int64_t lddw, float* db, int accumulate,
                         hipStream_t st) {
  GemmArgs g{};
  g.M = N; g.N = K; g.K = M;
  g.A = dY; g.a_rs = 1; g.a_cs = ldg;       // A(m=n, k=r) = dY[r][n]
  g.B = X; g.b_rs = ldx; g.b_cs = 1;        // B(k=r, n=k') = X[r][k']
  g.C = dW; g.ldc = lddw; g.accumulate = accumulate;
  int rc = gemm_launch(EPI_DW, g, st);
  if (rc || !db) return rc;
  hipLaunchKernelGGL(colsum_kernel, dim3((N + 63) / 64), dim3(kWG), 0, st, dY, M, N, ldg, db,
                     accumulate);
  return check_launch("colsum_kernel");
}

}  // namespace smi
