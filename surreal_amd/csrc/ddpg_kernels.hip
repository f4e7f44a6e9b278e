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
#include "smi_device.hpp"
#include "smi_internal.hpp"

namespace smi {

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

}  // namespace smi
