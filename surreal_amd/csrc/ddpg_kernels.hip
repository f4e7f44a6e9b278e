// ddpg_kernels.hip — elementwise/reduction pieces of DDPGLearner._optimize
// (surreal/learner/ddpg.py:244-352) and _target_update (ddpg.py:403-428);
// the dense layers run on linear_kernels.hip.
//
//   mse_grad        critic loss nn.MSELoss()(Q, y): loss, dQ = 2 (Q - y) / n
//   neg_mean_grad   actor loss -Q(s, mu(s)).mean(): loss, dQ = -1 / n
//   tanh_backward   d/dz tanh(z) = 1 - tanh(z)^2 (actor output layer)
//   copy_cols       write the action block of the critic's concat input
//   soft_update     target <- tau * src + (1 - tau) * target
//   ddpg_stats      action_norm, rewards, Q_target, Q_policy means (ddpg.py:335-345)
//   layernorm       the use_layernorm=True blocks of ActorNetworkX / CriticNetworkX
//                   (builders.py:41-48,65-75: Linear -> ReLU -> L.LayerNorm(1)),
//                   forward and backward (dx through the ReLU, dgamma, dbeta)
#include "smi_device.hpp"
#include "smi_internal.hpp"

namespace smi {

constexpr int kGatherMax = 16;      // segments per copy_gather launch

__global__ void __launch_bounds__(kWG)
mse_grad_kernel(const float* __restrict__ q, int64_t qs, const float* __restrict__ y, int64_t n,
                float* __restrict__ dq, float* loss) {
  __shared__ double scr[kNW];
  const float inv = 1.f / (float)n;
  double a = 0.0;
  for (int64_t i = threadIdx.x; i < n; i += kWG) {
    const float d = q[i * qs] - y[i];
    dq[i] = inv * (2.f * d);
    a += (double)(d * d);
  }
  a = block_sum_d(a, scr);
  if (threadIdx.x == 0 && loss) loss[0] = (float)(a / (double)n);
}

__global__ void __launch_bounds__(kWG)
neg_mean_grad_kernel(const float* __restrict__ q, int64_t qs, int64_t n, float* __restrict__ dq,
                     float* loss) {
  __shared__ double scr[kNW];
  const float g = -1.f / (float)n;
  double a = 0.0;
  for (int64_t i = threadIdx.x; i < n; i += kWG) {
    dq[i] = g;
    a += (double)q[i * qs];
  }
  a = block_sum_d(a, scr);
  if (threadIdx.x == 0 && loss) loss[0] = (float)(-a / (double)n);
}

__global__ void __launch_bounds__(kWG)
tanh_backward_kernel(const float* __restrict__ dy, int64_t ldg, const float* __restrict__ y,
                     int64_t ldy, int64_t rows, int cols, float* __restrict__ dz, int64_t ldz) {
  const int64_t total = rows * cols;
  for (int64_t e = (int64_t)blockIdx.x * kWG + threadIdx.x; e < total; e += (int64_t)gridDim.x * kWG) {
    const int64_t r = e / cols;
    const int c = (int)(e - r * cols);
    const float t = y[r * ldy + c];
    dz[r * ldz + c] = dy[r * ldg + c] * (1.f - t * t);
  }
}

__global__ void __launch_bounds__(kWG)
copy_cols_kernel(const float* __restrict__ src, int64_t lds, int64_t rows, int cols,
                 float* __restrict__ dst, int64_t ldd) {
  const int64_t total = rows * cols;
  for (int64_t e = (int64_t)blockIdx.x * kWG + threadIdx.x; e < total; e += (int64_t)gridDim.x * kWG) {
    const int64_t r = e / cols;
    const int c = (int)(e - r * cols);
    dst[r * ldd + c] = src[r * lds + c];
  }
}

// 16-byte grid-stride copy; dst may be pinned host memory mapped into the
// device address space (the publisher's D2H: a kernel on the side stream
// instead of an SDMA copy, so the host thread never blocks in the runtime)
__global__ void __launch_bounds__(kWG)
copy_bytes16_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst, int64_t n16) {
  for (int64_t i = (int64_t)blockIdx.x * kWG + threadIdx.x; i < n16; i += (int64_t)gridDim.x * kWG)
    dst[i] = src[i];
}

// up to kGatherMax device segments into one destination (the publisher's
// snapshot arena): blockIdx.y = segment, 16-byte body + 4-byte tail
struct GatherArgs {
  const char* src[kGatherMax]; int64_t off[kGatherMax]; int64_t nbytes[kGatherMax];
  char* dst;
};
__global__ void __launch_bounds__(kWG)
copy_gather_kernel(GatherArgs a) {
  const int s = blockIdx.y;
  const char* __restrict__ src = a.src[s];
  char* __restrict__ dst = a.dst + a.off[s];
  const int64_t n = a.nbytes[s], n16 = n >> 4;
  const int64_t t0 = (int64_t)blockIdx.x * kWG + threadIdx.x, ts = (int64_t)gridDim.x * kWG;
  for (int64_t i = t0; i < n16; i += ts)
    reinterpret_cast<uint4*>(dst)[i] = reinterpret_cast<const uint4*>(src)[i];
  for (int64_t i = (n16 << 2) + t0; i < (n >> 2); i += ts)
    reinterpret_cast<float*>(dst)[i] = reinterpret_cast<const float*>(src)[i];
}

__global__ void __launch_bounds__(kWG)
soft_update_kernel(float* __restrict__ t, const float* __restrict__ s, int64_t n, float tau) {
  for (int64_t i = (int64_t)blockIdx.x * kWG + threadIdx.x; i < n; i += (int64_t)gridDim.x * kWG)
    t[i] = tau * s[i] + (1.f - tau) * t[i];
}

// stats[0] action_norm = mean_r ||a_r||_2 ; [1] rewards mean ; [2] Q_target (y) mean ;
// [3] Q_policy mean
__global__ void __launch_bounds__(kWG)
ddpg_stats_kernel(const float* __restrict__ a, int64_t lda, int A, const float* __restrict__ r,
                  int64_t rs, const float* __restrict__ y, const float* __restrict__ q, int64_t qs,
                  int64_t n, float* stats) {
  __shared__ double scr[kNW];
  double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
  for (int64_t i = threadIdx.x; i < n; i += kWG) {
    float nn = 0.f;
    for (int j = 0; j < A; ++j) { const float v = a[i * lda + j]; nn += v * v; }
    s0 += (double)sqrtf(nn);
    s1 += (double)r[i * rs];
    s2 += (double)y[i];
    s3 += (double)q[i * qs];
  }
  s0 = block_sum_d(s0, scr); s1 = block_sum_d(s1, scr);
  s2 = block_sum_d(s2, scr); s3 = block_sum_d(s3, scr);
  if (threadIdx.x == 0) {
    stats[0] = (float)(s0 / n); stats[1] = (float)(s1 / n);
    stats[2] = (float)(s2 / n); stats[3] = (float)(s3 / n);
  }
}

static int grid_of(int64_t n) {
  int64_t g = (n + kWG - 1) / kWG;
  if (g < 1) g = 1;
  return (int)(g < 2048 ? g : 2048);
}

// ---------------------------------------------------------------- LayerNorm
// torchx's L.LayerNorm(1) normalises the last dimension; it is taken here as
// torch.nn.LayerNorm(n): biased variance, eps inside the square root, affine
// gamma / beta (torchx is not available: parity unpinned).
// One wave per row (n <= 64 * LN_MAXV), the row held in registers: mean, then
// the centred second moment (two passes over registers, no cancellation).
constexpr int LN_MAXV = 16;

__global__ void __launch_bounds__(kWG)
layernorm_fwd_kernel(const float* __restrict__ x, int64_t ldx, int64_t rows, int n,
                     const float* __restrict__ gamma, const float* __restrict__ beta, float eps,
                     float* __restrict__ y, int64_t ldy, float* __restrict__ mean,
                     float* __restrict__ rstd) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * (kWG / 64) + (threadIdx.x >> 6);
  if (r >= rows) return;
  const float* xr = x + r * ldx;
  float v[LN_MAXV];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < LN_MAXV; ++i) {
    const int c = lane + 64 * i;
    v[i] = c < n ? xr[c] : 0.f;
    s += v[i];
  }
  const float mu = wave_sum(s) / (float)n;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < LN_MAXV; ++i) {
    const int c = lane + 64 * i;
    const float d = v[i] - mu;
    q += c < n ? d * d : 0.f;
  }
  const float rs = 1.f / sqrtf(wave_sum(q) / (float)n + eps);
  float* yr = y + r * ldy;
#pragma unroll
  for (int i = 0; i < LN_MAXV; ++i) {
    const int c = lane + 64 * i;
    if (c < n) yr[c] = (v[i] - mu) * rs * gamma[c] + beta[c];
  }
  if (lane == 0) {
    mean[r] = mu;
    rstd[r] = rs;
  }
}

// dx = rstd (g - mean(g) - xhat mean(g xhat)), g = dy gamma, xhat = (x - mu) rstd,
// then through the ReLU that produced x (relu != 0: dx = 0 where x <= 0);
// per-block partials of dgamma = sum dy xhat and dbeta = sum dy ([nblk][2][n]),
// the block's waves combined in a fixed order
__global__ void __launch_bounds__(kWG)
layernorm_bwd_kernel(const float* __restrict__ dy, int64_t ldg, const float* __restrict__ x,
                     int64_t ldx, const float* __restrict__ mean, const float* __restrict__ rstd,
                     const float* __restrict__ gamma, int64_t rows, int n, int relu,
                     float* __restrict__ dx, int64_t lddx, float* __restrict__ part) {
  __shared__ float red[kWG / 64][2][64 * LN_MAXV];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float dg[LN_MAXV], db[LN_MAXV];
#pragma unroll
  for (int i = 0; i < LN_MAXV; ++i) dg[i] = db[i] = 0.f;
  for (int64_t r = (int64_t)blockIdx.x * (kWG / 64) + wave; r < rows;
       r += (int64_t)gridDim.x * (kWG / 64)) {
    const float mu = mean[r], rs = rstd[r];
    float xh[LN_MAXV], g[LN_MAXV];
    bool keep[LN_MAXV];
    float a = 0.f, b = 0.f;
#pragma unroll
    for (int i = 0; i < LN_MAXV; ++i) {
      const int c = lane + 64 * i;
      const bool ok = c < n;
      const float xv = ok ? x[r * ldx + c] : 0.f;
      const float d = ok ? dy[r * ldg + c] : 0.f;
      xh[i] = ok ? (xv - mu) * rs : 0.f;
      g[i] = ok ? d * gamma[c] : 0.f;
      a += g[i];
      b += g[i] * xh[i];
      dg[i] += d * xh[i];
      db[i] += d;
      keep[i] = !relu || xv > 0.f;
    }
    const float am = wave_sum(a) / (float)n, bm = wave_sum(b) / (float)n;
#pragma unroll
    for (int i = 0; i < LN_MAXV; ++i) {
      const int c = lane + 64 * i;
      if (c < n) dx[r * lddx + c] = keep[i] ? rs * (g[i] - am - xh[i] * bm) : 0.f;
    }
  }
#pragma unroll
  for (int i = 0; i < LN_MAXV; ++i) {
    red[wave][0][lane + 64 * i] = dg[i];
    red[wave][1][lane + 64 * i] = db[i];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < n; c += kWG) {
    float sg = 0.f, sb = 0.f;
#pragma unroll
    for (int w = 0; w < kWG / 64; ++w) {
      sg += red[w][0][c];
      sb += red[w][1][c];
    }
    part[((int64_t)blockIdx.x * 2) * n + c] = sg;
    part[((int64_t)blockIdx.x * 2 + 1) * n + c] = sb;
  }
}

// dgamma / dbeta: block partials summed in block order
__global__ void __launch_bounds__(kWG)
layernorm_param_grad_kernel(const float* __restrict__ part, int nb, int n, float* dgamma,
                            float* dbeta) {
  const int c = blockIdx.x * kWG + threadIdx.x;
  if (c >= 2 * n) return;
  const int which = c / n, col = c - which * n;
  float s = 0.f;
  for (int b = 0; b < nb; ++b) s += part[((int64_t)b * 2 + which) * n + col];
  (which ? dbeta : dgamma)[col] = s;
}

int launch_mse_grad(const float* q, int64_t qs, const float* y, int64_t n, float* dq, float* loss,
                    hipStream_t st) {
  hipLaunchKernelGGL(mse_grad_kernel, dim3(1), dim3(kWG), 0, st, q, qs, y, n, dq, loss);
  return check_launch("mse_grad_kernel");
}
int launch_neg_mean_grad(const float* q, int64_t qs, int64_t n, float* dq, float* loss,
                         hipStream_t st) {
  hipLaunchKernelGGL(neg_mean_grad_kernel, dim3(1), dim3(kWG), 0, st, q, qs, n, dq, loss);
  return check_launch("neg_mean_grad_kernel");
}
int launch_tanh_backward(const float* dy, int64_t ldg, const float* y, int64_t ldy, int64_t rows,
                         int cols, float* dz, int64_t ldz, hipStream_t st) {
  hipLaunchKernelGGL(tanh_backward_kernel, dim3(grid_of(rows * cols)), dim3(kWG), 0, st, dy, ldg,
                     y, ldy, rows, cols, dz, ldz);
  return check_launch("tanh_backward_kernel");
}
int launch_copy_cols(const float* src, int64_t lds, int64_t rows, int cols, float* dst,
                     int64_t ldd, hipStream_t st) {
  hipLaunchKernelGGL(copy_cols_kernel, dim3(grid_of(rows * cols)), dim3(kWG), 0, st, src, lds, rows,
                     cols, dst, ldd);
  return check_launch("copy_cols_kernel");
}
int launch_copy_bytes16(const void* src, void* dst, int64_t n16, hipStream_t st) {
  int64_t g = (n16 + kWG - 1) / kWG;
  if (g > 256) g = 256;
  if (g < 1) g = 1;
  hipLaunchKernelGGL(copy_bytes16_kernel, dim3((unsigned)g), dim3(kWG), 0, st,
                     reinterpret_cast<const uint4*>(src), reinterpret_cast<uint4*>(dst), n16);
  return check_launch("copy_bytes16_kernel");
}
int launch_copy_gather(void* dst, const void* const* srcs, const int64_t* offs,
                       const int64_t* nbytes, int n, hipStream_t st) {
  for (int b = 0; b < n; b += kGatherMax) {
    GatherArgs a{};
    a.dst = static_cast<char*>(dst);
    const int m = n - b < kGatherMax ? n - b : kGatherMax;
    int64_t mx = 0;
    for (int i = 0; i < m; ++i) {
      a.src[i] = static_cast<const char*>(srcs[b + i]);
      a.off[i] = offs[b + i];
      a.nbytes[i] = nbytes[b + i];
      mx = nbytes[b + i] > mx ? nbytes[b + i] : mx;
    }
    int64_t g = (mx / 16 + kWG - 1) / kWG;
    g = g < 1 ? 1 : (g > 64 ? 64 : g);
    hipLaunchKernelGGL(copy_gather_kernel, dim3((unsigned)g, (unsigned)m), dim3(kWG), 0, st, a);
    const int rc = check_launch("copy_gather_kernel");
    if (rc) return rc;
  }
  return SMI_OK;
}
int launch_soft_update(float* t, const float* s, int64_t n, float tau, hipStream_t st) {
  hipLaunchKernelGGL(soft_update_kernel, dim3(grid_of(n)), dim3(kWG), 0, st, t, s, n, tau);
  return check_launch("soft_update_kernel");
}
int launch_ddpg_stats(const float* a, int64_t lda, int A, const float* r, int64_t rs,
                      const float* y, const float* q, int64_t qs, int64_t n, float* stats,
                      hipStream_t st) {
  hipLaunchKernelGGL(ddpg_stats_kernel, dim3(1), dim3(kWG), 0, st, a, lda, A, r, rs, y, q, qs, n,
                     stats);
  return check_launch("ddpg_stats_kernel");
}

int launch_layernorm_fwd(const float* x, int64_t ldx, int64_t rows, int n, const float* gamma,
                         const float* beta, float eps, float* y, int64_t ldy, float* mean,
                         float* rstd, hipStream_t st) {
  if (n < 1 || n > 64 * LN_MAXV) return set_error(SMI_E_ARG, "layernorm: width must be in [1, 1024]");
  if (rows <= 0) return SMI_OK;
  const int64_t g = (rows + kWG / 64 - 1) / (kWG / 64);
  hipLaunchKernelGGL(layernorm_fwd_kernel, dim3((unsigned)g), dim3(kWG), 0, st, x, ldx, rows, n,
                     gamma, beta, eps, y, ldy, mean, rstd);
  return check_launch("layernorm_fwd_kernel");
}

int launch_layernorm_bwd(const float* dy, int64_t ldg, const float* x, int64_t ldx,
                         const float* mean, const float* rstd, const float* gamma, int64_t rows,
                         int n, int relu, float* dx, int64_t lddx, float* dgamma, float* dbeta,
                         hipStream_t st) {
  if (n < 1 || n > 64 * LN_MAXV) return set_error(SMI_E_ARG, "layernorm: width must be in [1, 1024]");
  int64_t nb = (rows + kWG / 64 - 1) / (kWG / 64);
  if (nb > 256) nb = 256;
  if (nb < 1) nb = 1;
  float* part = workspace_f32(nb * 2 * n);
  if (!part) return set_error(SMI_E_ARG, "layernorm: workspace unavailable");
  hipLaunchKernelGGL(layernorm_bwd_kernel, dim3((unsigned)nb), dim3(kWG), 0, st, dy, ldg, x, ldx,
                     mean, rstd, gamma, rows, n, relu, dx, lddx, part);
  RC_CHECK(check_launch("layernorm_bwd_kernel"));
  hipLaunchKernelGGL(layernorm_param_grad_kernel, dim3((2 * n + kWG - 1) / kWG), dim3(kWG), 0, st,
                     part, (int)nb, n, dgamma, dbeta);
  return check_launch("layernorm_param_grad_kernel");
}

}  // namespace smi

namespace smi {
// ---- batched parameter-noise acting (ddpg_agent.py:134-151,172-173) --------
// N agents, each with ITS OWN perturbed actor (param_noise.py:17-24 / 63-70):
// row i of x goes through the parameter set at params + i * pstride (the
// actor's flat layout, layer offsets o[0..5] = W1 b1 W2 b2 W3 b3), one
// workgroup per agent, every layer's input in LDS; output unit j of a layer
// is a wave's dot product (lanes over k, a fixed-order butterfly sum) plus
// its bias, then ReLU (hidden) or the output activation.  One launch for all
// N agents instead of N forwards.
struct Mlp3StackedArgs {
  const float* P; int64_t pstride;
  int64_t o[6];
  int in, h1, h2, out, act_out;
  const float* x; int64_t ldx;
  float* y; int64_t ldy;
};
constexpr int kMlp3MaxW = 1024;          // widest layer input / output

__device__ __forceinline__ void mlp3_layer(const float* __restrict__ W, const float* __restrict__ b,
                                           int K, int N, const float* __restrict__ a,
                                           float* __restrict__ o, int act) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int j = wave; j < N; j += kWG / 64) {
    const float* w = W + (int64_t)j * K;
    float s = 0.f;
    for (int k = lane; k < K; k += 64) s = fmaf(w[k], a[k], s);
    s = wave_sum(s);
    if (lane == 0) {
      float v = s + b[j];
      if (act == ACT_RELU) v = v > 0.f ? v : 0.f;
      else if (act == ACT_TANH) v = tanhf(v);
      o[j] = v;
    }
  }
}

__global__ void __launch_bounds__(kWG) mlp3_stacked_kernel(Mlp3StackedArgs a) {
  __shared__ float s0[kMlp3MaxW], s1[kMlp3MaxW], s2[kMlp3MaxW];
  const int i = blockIdx.x;
  const float* P = a.P + (int64_t)i * a.pstride;
  for (int k = threadIdx.x; k < a.in; k += kWG) s0[k] = a.x[(int64_t)i * a.ldx + k];
  __syncthreads();
  mlp3_layer(P + a.o[0], P + a.o[1], a.in, a.h1, s0, s1, ACT_RELU);
  __syncthreads();
  mlp3_layer(P + a.o[2], P + a.o[3], a.h1, a.h2, s1, s2, ACT_RELU);
  __syncthreads();
  mlp3_layer(P + a.o[4], P + a.o[5], a.h2, a.out, s2, s0, a.act_out);
  __syncthreads();
  for (int k = threadIdx.x; k < a.out; k += kWG) a.y[(int64_t)i * a.ldy + k] = s0[k];
}

int launch_mlp3_stacked(const float* P, int64_t pstride, const int64_t* o6, int in, int h1, int h2,
                        int out, int act_out, const float* x, int64_t ldx, int n, float* y,
                        int64_t ldy, hipStream_t st) {
  if (in < 1 || h1 < 1 || h2 < 1 || out < 1 || in > kMlp3MaxW || h1 > kMlp3MaxW ||
      h2 > kMlp3MaxW || out > kMlp3MaxW)
    return set_error(SMI_E_NOFIT, "mlp3_forward_stacked: layer widths must be in [1, 1024]");
  Mlp3StackedArgs a{P, pstride, {o6[0], o6[1], o6[2], o6[3], o6[4], o6[5]}, in, h1, h2, out,
                    act_out, x, ldx, y, ldy};
  hipLaunchKernelGGL(mlp3_stacked_kernel, dim3(n), dim3(kWG), 0, st, a);
  return check_launch("mlp3_stacked_kernel");
}
}  // namespace smi
