// ops_kernels.hip — elementwise / reduction kernels of the learner hot path and
// the standalone model ops behind the PPOModel / ZFilter / DiagGauss mirrors.
//
//   zfilter_apply / zfilter_colstats / zfilter_update   z_filter.py:44-79
//   reward_filter                                        reward_filter.py:18-56
//   diag_gauss                                           ppo_net.py:29-72
//   mlp_forward                                          ppo_net.py:253-315
//   moments                                              ppo.py:402-405,413-416
//   adam_clip                                            ppo.py:243-247 (torch Adam)
//   ddpg_target                                          ddpg.py:279-283
#include "smi_device.hpp"
#include "smi_internal.hpp"

namespace smi {

// ------------------------------------------------------------- ZFilter apply
// HBM-bound (8 B per element).  16-byte loads/stores; the column of each of a
// float4's four elements is tracked incrementally (no per-element modulo).
__global__ void __launch_bounds__(kWG)
zfilter_apply_kernel(const float* __restrict__ x, float* __restrict__ out, int64_t n, int dim,
                     const float* sum, const float* sumsq, const float* count, float eps) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* zm = sm;
  float* zs = sm + round4(dim);
  zfilter_colstats(sum, sumsq, count, eps, dim, zm, zs);
  __syncthreads();
  const bool vec = ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(out)) & 15) == 0;
  const int64_t n4 = vec ? (n >> 2) : 0;
  const int64_t stride = (int64_t)gridDim.x * kWG;
  const float4* x4 = reinterpret_cast<const float4*>(x);
  float4* o4 = reinterpret_cast<float4*>(out);
  for (int64_t i = (int64_t)blockIdx.x * kWG + threadIdx.x; i < n4; i += stride) {
    const float4 v = x4[i];
    int c = (int)((i << 2) % dim);
    float r[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float y = (r[j] - zm[c]) / zs[c];
      r[j] = fminf(fmaxf(y, -5.f), 5.f);
      c = (c + 1 == dim) ? 0 : c + 1;
    }
    o4[i] = float4{r[0], r[1], r[2], r[3]};
  }
  for (int64_t i = (n4 << 2) + (int64_t)blockIdx.x * kWG + threadIdx.x; i < n; i += stride) {
    const int c = (int)(i % dim);
    const float y = (x[i] - zm[c]) / zs[c];
    out[i] = fminf(fmaxf(y, -5.f), 5.f);
  }
}

// ------------------------------------------------ ZFilter column statistics
// Column sums and sums of squares over `rows` strided rows (HBM-bound, 4 B per
// element).  A workgroup covers CB = min(dim, 256) columns with RP = 256/CB row
// lanes, so for contiguous rows (stride == dim) one wave-instruction reads 256
// consecutive bytes; 8 independent loads per thread are kept in flight.
// Partial sums go to `part` [gridDim.y][2][dim], reduced in a fixed order by
// the finisher (deterministic).
__global__ void __launch_bounds__(kWG)
colstats_partial_kernel(const float* __restrict__ x, int64_t rows, int dim, int64_t stride,
                        float* __restrict__ part) {
  __shared__ float s1[kWG], s2[kWG];
  const int CB = dim < kWG ? dim : kWG;
  const int RP = kWG / CB;
  const int t = threadIdx.x;
  const int rl = t / CB, cl = t - rl * CB;
  const int c = blockIdx.x * CB + cl;
  const bool active = rl < RP && c < dim;
  float a1 = 0.f, a2 = 0.f;
  if (active) {
    // this workgroup's contiguous row range (a wave walks consecutive memory)
    const int64_t per = (rows + gridDim.y - 1) / gridDim.y;
    const int64_t r_lo = (int64_t)blockIdx.y * per;
    const int64_t r_hi = min(rows, r_lo + per);
    int64_t r = r_lo + rl;
    for (; r + 7 * RP < r_hi; r += 8 * RP) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = x[(r + u * RP) * stride + c];
#pragma unroll
      for (int u = 0; u < 8; ++u) { a1 += v[u]; a2 += v[u] * v[u]; }
    }
    for (; r < r_hi; r += RP) {
      const float v = x[r * stride + c];
      a1 += v;
      a2 += v * v;
    }
  }
  s1[t] = a1;
  s2[t] = a2;
  __syncthreads();
  if (rl == 0 && c < dim) {
    float t1 = 0.f, t2 = 0.f;
    for (int w = 0; w < RP; ++w) { t1 += s1[w * CB + cl]; t2 += s2[w * CB + cl]; }
    part[((int64_t)blockIdx.y * 2) * dim + c] = t1;
    part[((int64_t)blockIdx.y * 2 + 1) * dim + c] = t2;
  }
}

// finisher: one workgroup per column reduces the partials (fixed order);
// mode 0 -> write sums; mode 1 -> add into running buffers and count
__global__ void __launch_bounds__(kWG)
colstats_finish_kernel(const float* __restrict__ part, int nparts, int dim, int64_t rows,
                       int mode, float* out_sum, float* out_sumsq, float* count) {
  __shared__ double scr[kNW];
  const int c = blockIdx.x;
  float t1 = 0.f, t2 = 0.f;
  for (int p = threadIdx.x; p < nparts; p += kWG) {
    t1 += part[((int64_t)p * 2) * dim + c];
    t2 += part[((int64_t)p * 2 + 1) * dim + c];
  }
  const float s1 = block_sum_f(t1, scr);
  const float s2 = block_sum_f(t2, scr);
  if (threadIdx.x == 0) {
    if (mode == 0) {
      out_sum[c] = s1;
      out_sumsq[c] = s2;
    } else {
      out_sum[c] += s1;      // running_sum += torch.sum(x, 0)   (z_filter.py:54)
      out_sumsq[c] += s2;    // running_sumsq += torch.sum(x*x, 0) (z_filter.py:55)
      if (c == 0) count[0] += (float)rows;                          // :56
    }
  }
}

// Single-pass variant for small inputs: one workgroup, no partial buffer.
__global__ void __launch_bounds__(kWG)
colstats_small_kernel(const float* __restrict__ x, int64_t rows, int dim, int64_t stride,
                      int mode, float* out_sum, float* out_sumsq, float* count) {
  __shared__ float s1[kNW][64], s2[kNW][64];
  const int rl = threadIdx.x >> 6, cl = threadIdx.x & 63;
  for (int c0 = 0; c0 < dim; c0 += 64) {
    const int c = c0 + cl;
    float a1 = 0.f, a2 = 0.f;
    if (c < dim)
      for (int64_t r = rl; r < rows; r += kNW) {
        const float v = x[r * stride + c];
        a1 += v;
        a2 += v * v;
      }
    s1[rl][cl] = a1; s2[rl][cl] = a2;
    __syncthreads();
    if (rl == 0 && c < dim) {
      float t1 = 0.f, t2 = 0.f;
      for (int w = 0; w < kNW; ++w) { t1 += s1[w][cl]; t2 += s2[w][cl]; }
      if (mode == 0) { out_sum[c] = t1; out_sumsq[c] = t2; }
      else { out_sum[c] += t1; out_sumsq[c] += t2; }
    }
    __syncthreads();
  }
  if (mode == 1 && threadIdx.x == 0) count[0] += (float)rows;
}

// ------------------------------------------------------------- RewardFilter
// rewards *= reward_scale (ppo.py:452); then, by mode bits,
//   1: forward  — clamp((r - mean)/max(sqrt(sumsq/count - mean^2), eps), +-5)
//      with the running stats from BEFORE this call's update (reward_filter.py:44-56)
//   2: update   — count += n, running_sum += sum(r), running_sumsq = sum(r*r)
//      (the reference's '=' instead of '+=' at reward_filter.py:42 is kept)
//   4: partial  — instead of updating, write {sum(r), sum(r*r), n} (fp64) to
//      out3: a data-parallel learner all-reduces them and commits the global
//      sums with reward_filter_commit_kernel, so every rank's filter equals
//      the one a single process would hold after the global batch
__global__ void __launch_bounds__(kWG)
reward_filter_kernel(float* __restrict__ r, int64_t n, float scale, int mode,
                     float* rsum, float* rsumsq, float* rcount, float eps, double* out3) {
  __shared__ double scr[kNW];
  float mean = 0.f, sd = 1.f;
  if (mode & 1) {
    const float cnt = rcount[0];
    mean = rsum[0] / cnt;
    const float v = rsumsq[0] / cnt - mean * mean;
    sd = sqrtf(v);
    sd = sd < eps ? eps : sd;
  }
  double a1 = 0.0, a2 = 0.0;
  for (int64_t i = threadIdx.x; i < n; i += kWG) {
    const float x = r[i] * scale;
    a1 += (double)x;
    a2 += (double)(x * x);
    if (mode & 1) {
      const float y = (x - mean) / sd;
      r[i] = fminf(fmaxf(y, -5.f), 5.f);
    } else {
      r[i] = x;
    }
  }
  if (mode & 6) {
    const double t1 = block_sum_d(a1, scr);
    const double t2 = block_sum_d(a2, scr);
    if (threadIdx.x == 0) {
      if (mode & 4) {
        out3[0] = t1; out3[1] = t2; out3[2] = (double)n;
      } else {
        rcount[0] = rcount[0] + (float)n;
        rsum[0] = rsum[0] + (float)t1;
        rsumsq[0] = (float)t2;
      }
    }
  }
}

// the update of mode 2 from (all-reduced) sums {sum, sumsq, n}
__global__ void reward_filter_commit_kernel(const double* __restrict__ s3, float* rsum,
                                            float* rsumsq, float* rcount) {
  if (threadIdx.x == 0) {
    rcount[0] = rcount[0] + (float)s3[2];
    rsum[0] = rsum[0] + (float)s3[0];
    rsumsq[0] = (float)s3[1];
  }
}

// ------------------------------------------------------------ DiagGauss ops
// HBM-bound: a tile of DG_R rows of actions (A floats), prob0 and prob1 (2A
// floats each) is staged through LDS with 16-byte coalesced loads (the tile is
// contiguous in each array), then one thread per row forms the sums from LDS
// with odd row strides (bank-conflict free); outputs are written coalesced.
constexpr int DG_R = kWG;

__device__ __forceinline__ void stage_rows(const float* __restrict__ src, int64_t r0, int nrows,
                                           int w, float* __restrict__ dst, int ldd) {
  const int n = nrows * w;
  const float* g = src + r0 * w;
  if (((reinterpret_cast<uintptr_t>(g)) & 15) == 0 && (w & 3) == 0) {
    const int w4 = w >> 2;
    const float4* g4 = reinterpret_cast<const float4*>(g);
    for (int e = threadIdx.x; e < (n >> 2); e += kWG) {
      const float4 v = g4[e];
      const int r = e / w4, c = (e - r * w4) << 2;
      float* d = dst + r * ldd + c;
      d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
    }
  } else {
    for (int e = threadIdx.x; e < n; e += kWG) {
      const int r = e / w, c = e - r * w;
      dst[r * ldd + c] = g[e];
    }
  }
}

__global__ void __launch_bounds__(kWG)
diag_gauss_kernel(const float* __restrict__ a, const float* __restrict__ p0,
                  const float* __restrict__ p1, int64_t rows, int A, float c_ll, float c_ent,
                  float* loglik, float* lik, float* kl, float* ent) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int lda = A | 1, ldp = (2 * A) | 1;
  const bool need_a = loglik || lik;
  const bool need_p1 = kl && p1;
  float* sa = sm;
  float* s0 = sa + DG_R * lda;
  float* s1 = s0 + DG_R * ldp;
  const int64_t ntiles = (rows + DG_R - 1) / DG_R;
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int64_t r0 = tile * DG_R;
    const int nr = (int)min((int64_t)DG_R, rows - r0);
    __syncthreads();
    if (need_a) stage_rows(a, r0, nr, A, sa, lda);
    stage_rows(p0, r0, nr, 2 * A, s0, ldp);
    if (need_p1) stage_rows(p1, r0, nr, 2 * A, s1, ldp);
    __syncthreads();
    const int r = threadIdx.x;
    if (r >= nr) continue;
    const float* q0 = s0 + r * ldp;
    float lsum = 0.f;
    for (int j = 0; j < A; ++j) lsum += logf(q0[A + j]);
    if (need_a) {
      const float* ar = sa + r * lda;
      float sq = 0.f;
      for (int j = 0; j < A; ++j) {
        const float u = (ar[j] - q0[j]) / q0[A + j];
        sq += u * u;
      }
      const float ll = (-0.5f * sq - c_ll) - lsum;
      if (loglik) loglik[r0 + r] = ll;
      if (lik) lik[r0 + r] = fmaxf(expf(ll), 1e-5f);
    }
    if (need_p1) {
      const float* q1 = s1 + r * ldp;
      float k1 = 0.f, k2 = 0.f;
      for (int j = 0; j < A; ++j) {
        k1 += logf(q1[A + j] / q0[A + j]);
        const float d = q0[j] - q1[j];
        k2 += (q0[A + j] * q0[A + j] + d * d) / (2.f * (q1[A + j] * q1[A + j]));
      }
      kl[r0 + r] = (k1 + k2) - 0.5f * (float)A;
    }
    if (ent) ent[r0 + r] = 0.5f * lsum + c_ent;
  }
}

// Row-direct variant for A <= 8 (every BASELINE config): no LDS, no barriers.
// Each thread owns whole rows and reads them with the widest aligned vector
// loads (a row is 4A / 8A / 8A bytes); consecutive lanes read consecutive
// rows, so the lines a wave touches are fully consumed from L1 by its next
// vector loads.  U rows per thread are loaded before any is used.
template <int W>
struct VecT;
template <> struct VecT<1> { typedef float T; };
template <> struct VecT<2> { typedef float2 T; };
template <> struct VecT<4> { typedef float4 T; };

template <int N, int W>
__device__ __forceinline__ void load_row(const float* __restrict__ src, float (&out)[N]) {
  typedef typename VecT<W>::T V;
  const V* s = reinterpret_cast<const V*>(src);
#pragma unroll
  for (int i = 0; i < N / W; ++i) {
    const V v = s[i];
    const float* f = reinterpret_cast<const float*>(&v);
#pragma unroll
    for (int k = 0; k < W; ++k) out[i * W + k] = f[k];
  }
}

template <int A>
__global__ void __launch_bounds__(kWG)
diag_gauss_rows_kernel(const float* __restrict__ a, const float* __restrict__ p0,
                       const float* __restrict__ p1, int64_t rows, float c_ll, float c_ent,
                       float* loglik, float* lik, float* kl, float* ent) {
  constexpr int WA = (A % 4 == 0) ? 4 : (A % 2 == 0) ? 2 : 1;
  constexpr int WP = (A % 2 == 0) ? 4 : 2;
  constexpr int U = 2;
  const bool need_a = loglik || lik;
  const bool need_p1 = kl && p1;
  const int64_t nth = (int64_t)gridDim.x * kWG;
  for (int64_t r0 = (int64_t)blockIdx.x * kWG + threadIdx.x; r0 < rows; r0 += U * nth) {
    float ar[U][A], q0[U][2 * A], q1[U][2 * A];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      int64_t r = r0 + u * nth;
      r = r < rows ? r : rows - 1;                   // clamped: every load is unconditional
      load_row<2 * A, WP>(p0 + r * 2 * A, q0[u]);
      if (need_a) load_row<A, WA>(a + r * A, ar[u]);
      if (need_p1) load_row<2 * A, WP>(p1 + r * 2 * A, q1[u]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t r = r0 + u * nth;
      if (r >= rows) break;
      float lsum = 0.f;
#pragma unroll
      for (int j = 0; j < A; ++j) lsum += logf(q0[u][A + j]);
      if (need_a) {
        float sq = 0.f;
#pragma unroll
        for (int j = 0; j < A; ++j) {
          const float z = (ar[u][j] - q0[u][j]) / q0[u][A + j];
          sq += z * z;
        }
        const float ll = (-0.5f * sq - c_ll) - lsum;
        if (loglik) loglik[r] = ll;
        if (lik) lik[r] = fmaxf(expf(ll), 1e-5f);
      }
      if (need_p1) {
        float k1 = 0.f, k2 = 0.f;
#pragma unroll
        for (int j = 0; j < A; ++j) {
          k1 += logf(q1[u][A + j] / q0[u][A + j]);
          const float d = q0[u][j] - q1[u][j];
          k2 += (q0[u][A + j] * q0[u][A + j] + d * d) / (2.f * (q1[u][A + j] * q1[u][A + j]));
        }
        kl[r] = (k1 + k2) - 0.5f * (float)A;
      }
      if (ent) ent[r] = 0.5f * lsum + c_ent;
    }
  }
}

// -------------------------------------------------------------- MLP forward
struct MlpFwdArgs {
  const float* params; int in, h1, h2, out, act, lv;
  const float* x; int64_t rows, stride;
  int use_zf; const float *zsum, *zsumsq, *zcount; float zeps;
  float* y; int params_in_lds;
};

__global__ void __launch_bounds__(kWG)
mlp_forward_kernel(MlpFwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const MlpLayout L = mlp_layout(a.in, a.h1, a.h2, a.out, a.lv);
  const int ldX = pad_ld(a.in), ldH1 = pad_ld(a.h1), ldH2 = pad_ld(a.h2), ldO = pad_small(a.out);
  float* zm = sm;
  float* zs = zm + round4(a.in);
  float* X0 = zs + round4(a.in);
  float* H1 = X0 + kRT * ldX;
  float* H2 = H1 + kRT * ldH1;
  float* OUT = H2 + kRT * ldH2;
  float* P = OUT + kRT * ldO;
  if (a.use_zf) zfilter_colstats(a.zsum, a.zsumsq, a.zcount, a.zeps, a.in, zm, zs);
  MlpView V;
  if (a.params_in_lds) { mlp_load_lds(L, a.params, P); V = view_padded(L, P); }
  else V = view_flat(L, a.params);
  for (int e = threadIdx.x; e < kRT * (ldH1 + ldH2 + ldO); e += kWG) H1[e] = 0.f;
  __syncthreads();
  const int ntiles = (int)((a.rows + kRT - 1) / kRT);
  const int ocols = a.lv ? 2 * a.out : a.out;
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int64_t r0 = (int64_t)tile * kRT;
    const int nr = (int)min((int64_t)kRT, a.rows - r0);
    load_obs_tile(a.x + r0 * a.stride, a.stride, nr, a.in, a.use_zf ? zm : nullptr, zs, X0, ldX);
    __syncthreads();
    dense_fwd<ACT_RELU>(X0, ldX, V.W1, V.ld1, V.b1, a.in, a.h1, H1, ldH1);
    __syncthreads();
    dense_fwd<ACT_RELU>(H1, ldH1, V.W2, V.ld2, V.b2, a.h1, a.h2, H2, ldH2);
    __syncthreads();
    if (a.act == ACT_TANH) dense_fwd<ACT_TANH>(H2, ldH2, V.W3, V.ld3, V.b3, a.h2, a.out, OUT, ldO);
    else dense_fwd<ACT_NONE>(H2, ldH2, V.W3, V.ld3, V.b3, a.h2, a.out, OUT, ldO);
    __syncthreads();
    for (int e = threadIdx.x; e < nr * ocols; e += kWG) {
      const int r = e / ocols, j = e - r * ocols;
      const float v = j < a.out ? OUT[r * ldO + j] : expf(V.lv[j - a.out]);
      a.y[(r0 + r) * ocols + j] = v;
    }
    __syncthreads();
  }
}

// -------------------------------------------------------------- moments
// (sum, sumsq) of x in fp64: grid-stride partials with 16-byte loads, then a
// one-workgroup fixed-order finish (deterministic); or, given partials, only
// the finish.
__global__ void __launch_bounds__(kWG)
moments_partial_kernel(const float* __restrict__ x, int64_t n, double* __restrict__ part) {
  __shared__ double scr[kNW];
  double a1 = 0.0, a2 = 0.0;
  const int64_t stride = (int64_t)gridDim.x * kWG;
  const bool vec = (reinterpret_cast<uintptr_t>(x) & 15) == 0;
  const int64_t n4 = vec ? (n >> 2) : 0;
  const float4* x4 = reinterpret_cast<const float4*>(x);
  int64_t i = (int64_t)blockIdx.x * kWG + threadIdx.x;
  for (; i + stride < n4; i += 2 * stride) {
    const float4 u = x4[i], w = x4[i + stride];
    const float e[8] = {u.x, u.y, u.z, u.w, w.x, w.y, w.z, w.w};
#pragma unroll
    for (int j = 0; j < 8; ++j) { const double d = (double)e[j]; a1 += d; a2 += d * d; }
  }
  for (; i < n4; i += stride) {
    const float4 u = x4[i];
    const float e[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) { const double d = (double)e[j]; a1 += d; a2 += d * d; }
  }
  for (int64_t k = (n4 << 2) + (int64_t)blockIdx.x * kWG + threadIdx.x; k < n; k += stride) {
    const double d = (double)x[k];
    a1 += d;
    a2 += d * d;
  }
  const double t1 = block_sum_d(a1, scr);
  const double t2 = block_sum_d(a2, scr);
  if (threadIdx.x == 0) { part[2 * blockIdx.x] = t1; part[2 * blockIdx.x + 1] = t2; }
}

__global__ void __launch_bounds__(kWG)
moments_kernel(const float* __restrict__ x, int64_t n, const double* partials, int np,
               double* out) {
  __shared__ double scr[kNW];
  double a1 = 0.0, a2 = 0.0;
  if (partials && np > 0) {
    for (int i = threadIdx.x; i < np; i += kWG) { a1 += partials[2 * i]; a2 += partials[2 * i + 1]; }
  } else {
    for (int64_t i = threadIdx.x; i < n; i += kWG) {
      const double v = (double)x[i];
      a1 += v;
      a2 += v * v;
    }
  }
  const double t1 = block_sum_d(a1, scr);
  const double t2 = block_sum_d(a2, scr);
  if (threadIdx.x == 0) { out[0] = t1; out[1] = t2; out[2] = (double)n; }
}

// ||g||^2 partials in fp64 (clip_grad_norm_'s norm), 16-byte loads.
__global__ void __launch_bounds__(kWG)
sumsq_partial_kernel(const float* __restrict__ g, int64_t n, float clip_value, double* part) {
  __shared__ double scr[kNW];
  double a = 0.0;
  const int64_t stride = (int64_t)gridDim.x * kWG;
  const bool vec = (reinterpret_cast<uintptr_t>(g) & 15) == 0;
  const int64_t n4 = vec ? (n >> 2) : 0;
  const float4* g4 = reinterpret_cast<const float4*>(g);
  for (int64_t i = (int64_t)blockIdx.x * kWG + threadIdx.x; i < n4; i += stride) {
    const float4 u = g4[i];
    const float e[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float gi = e[j];
      if (clip_value > 0.f) gi = fminf(fmaxf(gi, -clip_value), clip_value);
      a += (double)gi * (double)gi;
    }
  }
  for (int64_t i = (n4 << 2) + (int64_t)blockIdx.x * kWG + threadIdx.x; i < n; i += stride) {
    float gi = g[i];
    if (clip_value > 0.f) gi = fminf(fmaxf(gi, -clip_value), clip_value);
    a += (double)gi * (double)gi;
  }
  a = block_sum_d(a, scr);
  if (threadIdx.x == 0) part[blockIdx.x] = a;
}

struct AdamCoef {
  float coef, wd, w1, beta2, w2, eps, step_size, bc2_sqrt, clip_value;
};

__device__ __forceinline__ void adam_elem(float& p, float g, float& m, float& v, const AdamCoef& k) {
  if (k.clip_value > 0.f) g = fminf(fmaxf(g, -k.clip_value), k.clip_value);   // clip_grad_value_
  g = g * k.coef;
  if (k.wd != 0.f) g = g + k.wd * p;
  m = m + k.w1 * (g - m);                      // m.lerp_(g, 1 - beta1)
  v = v * k.beta2 + (k.w2 * g) * g;            // v.mul_(b2).addcmul_(g, g, 1 - b2)
  const float denom = sqrtf(v) / k.bc2_sqrt + k.eps;
  p = p + (-k.step_size) * (m / denom);
}

// torch.optim.Adam (single-tensor path) on a flat buffer, after the optional
// clip_grad_norm_ coefficient.  HBM-bound: 28 B per parameter, 16-byte loads
// and stores of p, g, m, v.  NT bit 0: nontemporal stores of p, m, v; bit 1:
// nontemporal loads (streams touched once per launch at sweep sizes).
template <typename T>
__device__ __forceinline__ T adam_ld(const T* p, int nt) {
  return nt ? __builtin_nontemporal_load(p) : *p;
}
template <typename T>
__device__ __forceinline__ void adam_st(T* p, T v, int nt) {
  if (nt) __builtin_nontemporal_store(v, p); else *p = v;
}
__device__ __forceinline__ float4 adam_ld4(const float4* p, int nt) {
  if (!nt) return *p;
  const f32x4 u = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p));
  return float4{u[0], u[1], u[2], u[3]};
}
__device__ __forceinline__ void adam_st4(float4* p, float4 v, int nt) {
  if (!nt) { *p = v; return; }
  __builtin_nontemporal_store(f32x4{v.x, v.y, v.z, v.w}, reinterpret_cast<f32x4*>(p));
}

template <int NT>
__global__ void __launch_bounds__(kWG)
adam_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
            float* __restrict__ v, int64_t n, int* step, const float* lr_ptr, float beta1,
            float beta2, float eps, float wd, float max_norm, float clip_value, const double* part,
            int np, const int* skip, float* norm_out) {
  constexpr int NS = NT & 1, NL = (NT >> 1) & 1;
  if (skip && skip[0] != 0) return;
  __shared__ float s_coef;
  __shared__ int s_t;
  __shared__ double s_red[kNW];
  double s = 0.0;
  if (part)
    for (int i = threadIdx.x; i < np; i += kWG) s += part[i];
  s = block_sum_d(s, s_red);
  if (threadIdx.x == 0) {
    const float norm = (float)sqrt(s);
    float coef = 1.f;
    if (max_norm > 0.f) {
      const float cc = max_norm / (norm + 1e-6f);
      coef = cc < 1.f ? cc : 1.f;
    }
    s_coef = coef;
    s_t = step[0] + 1;
    if (blockIdx.x == 0 && norm_out) norm_out[0] = norm;
  }
  __syncthreads();
  const int t = s_t;
  const double bc1 = 1.0 - pow((double)beta1, (double)t);
  const double bc2 = 1.0 - pow((double)beta2, (double)t);
  AdamCoef k;
  k.coef = s_coef; k.wd = wd; k.beta2 = beta2; k.eps = eps; k.clip_value = clip_value;
  k.step_size = (float)((double)lr_ptr[0] / bc1);
  k.bc2_sqrt = (float)sqrt(bc2);
  k.w1 = (float)(1.0 - (double)beta1);
  k.w2 = (float)(1.0 - (double)beta2);
  const int64_t stride = (int64_t)gridDim.x * kWG;
  const bool vec = ((reinterpret_cast<uintptr_t>(p) | reinterpret_cast<uintptr_t>(g) |
                     reinterpret_cast<uintptr_t>(m) | reinterpret_cast<uintptr_t>(v)) & 15) == 0;
  const int64_t n4 = vec ? (n >> 2) : 0;
  float4* p4 = reinterpret_cast<float4*>(p);
  const float4* g4 = reinterpret_cast<const float4*>(g);
  float4* m4 = reinterpret_cast<float4*>(m);
  float4* v4 = reinterpret_cast<float4*>(v);
  int64_t i = (int64_t)blockIdx.x * kWG + threadIdx.x;
  for (; i < n4; i += stride) {
    float4 pp = adam_ld4(p4 + i, NL), mm = adam_ld4(m4 + i, NL), vv = adam_ld4(v4 + i, NL);
    const float4 gg = adam_ld4(g4 + i, NL);
    adam_elem(pp.x, gg.x, mm.x, vv.x, k);
    adam_elem(pp.y, gg.y, mm.y, vv.y, k);
    adam_elem(pp.z, gg.z, mm.z, vv.z, k);
    adam_elem(pp.w, gg.w, mm.w, vv.w, k);
    adam_st4(p4 + i, pp, NS); adam_st4(m4 + i, mm, NS); adam_st4(v4 + i, vv, NS);
  }
  for (int64_t i = (n4 << 2) + (int64_t)blockIdx.x * kWG + threadIdx.x; i < n; i += stride) {
    float pi = adam_ld(p + i, NL), mi = adam_ld(m + i, NL), vi = adam_ld(v + i, NL);
    adam_elem(pi, adam_ld(g + i, NL), mi, vi, k);
    adam_st(p + i, pi, NS); adam_st(m + i, mi, NS); adam_st(v + i, vi, NS);
  }
}

__global__ void step_inc_kernel(int* step, const int* skip) {
  if (skip && skip[0] != 0) return;
  step[0] += 1;
}

// ------------------------------------------------------------- DDPG target
__global__ void __launch_bounds__(kWG)
ddpg_target_kernel(const float* __restrict__ r, const float* __restrict__ d,
                   const float* __restrict__ q, const float* __restrict__ q2, int64_t n,
                   float gn, float* __restrict__ y) {
  for (int64_t i = (int64_t)blockIdx.x * kWG + threadIdx.x; i < n; i += (int64_t)gridDim.x * kWG) {
    const float nd = 1.f - d[i];
    float v = r[i] + (gn * q[i]) * nd;     // r + gamma^n * Q' * (1 - done)
    if (q2) {
      const float v2 = r[i] + (gn * q2[i]) * nd;
      v = fminf(v, v2);                       // torch.min(y, y2)
    }
    y[i] = v;
  }
}

static int grid_for(int64_t n, int cap = 2048) {
  int64_t g = (n + kWG - 1) / kWG;
  if (g < 1) g = 1;
  return (int)(g < cap ? g : cap);
}

// ============================================================ launchers
int launch_zfilter_apply(const float* x, float* out, int64_t rows, int dim, const float* s,
                         const float* sq, const float* cnt, float eps, hipStream_t st) {
  const int64_t n = rows * dim;
  if (n == 0) return SMI_OK;
  hipLaunchKernelGGL(zfilter_apply_kernel, dim3(grid_for((n + 3) / 4)), dim3(kWG),
                     (size_t)(2 * round4(dim) * 4), st, x, out, n, dim, s, sq, cnt, eps);
  return check_launch("zfilter_apply_kernel");
}

// scratch for colstats partials: caller-provided workspace is avoided by
// bounding the partial count; the partial buffer lives in a static device
// allocation made once at library load (see capi.cpp: smi_workspace()).
float* workspace_f32(int64_t nfloats);

int launch_colstats(const float* x, int64_t rows, int dim, int64_t stride, int mode,
                    float* osum, float* osq, float* cnt, hipStream_t st) {
  if (rows * (int64_t)dim <= (int64_t)1 << 16) {
    hipLaunchKernelGGL(colstats_small_kernel, dim3(1), dim3(kWG), 0, st, x, rows, dim, stride,
                       mode, osum, osq, cnt);
    return check_launch("colstats_small_kernel");
  }
  const int CB = dim < kWG ? dim : kWG;
  const int RP = kWG / CB;
  const int gx = (dim + CB - 1) / CB;
  int gy = (int)((rows + 8 * RP - 1) / (8 * RP));
  const int gy_cap = (2048 + gx - 1) / gx;
  if (gy > gy_cap) gy = gy_cap;
  if (gy < 1) gy = 1;
  float* part = workspace_f32((int64_t)gy * 2 * dim);
  hipLaunchKernelGGL(colstats_partial_kernel, dim3(gx, gy), dim3(kWG), 0, st, x, rows, dim,
                     stride, part);
  int rc = check_launch("colstats_partial_kernel");
  if (rc) return rc;
  hipLaunchKernelGGL(colstats_finish_kernel, dim3(dim), dim3(kWG), 0, st,
                     part, gy, dim, rows, mode, osum, osq, cnt);
  return check_launch("colstats_finish_kernel");
}

int launch_reward_filter(float* r, int64_t n, float scale, int use, float* s, float* sq,
                         float* c, float eps, double* out3, hipStream_t st) {
  hipLaunchKernelGGL(reward_filter_kernel, dim3(1), dim3(kWG), 0, st, r, n, scale, use, s, sq,
                     c, eps, out3);
  return check_launch("reward_filter_kernel");
}

int launch_reward_filter_commit(const double* s3, float* s, float* sq, float* c, hipStream_t st) {
  hipLaunchKernelGGL(reward_filter_commit_kernel, dim3(1), dim3(64), 0, st, s3, s, sq, c);
  return check_launch("reward_filter_commit_kernel");
}

int launch_diag_gauss(const float* a, const float* p0, const float* p1, int64_t rows, int A,
                      float* ll, float* lik, float* kl, float* ent, hipStream_t st) {
  const float c_ll = (float)(0.5 * log(2.0 * 3.141592653589793) * (double)A);
  const float c_ent = (float)(0.5 * log(2.0 * 3.141592653589793 * 2.718281828459045) * (double)A);
  if (rows <= 0) return SMI_OK;
  const bool al = ((reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(p0) |
                    reinterpret_cast<uintptr_t>(p1)) & 15) == 0;
  if (al && A >= 1 && A <= 8) {
    const int64_t want = (rows + 2 * kWG - 1) / (2 * kWG);
    const int grid = (int)(want < 8192 ? (want < 1 ? 1 : want) : 8192);
#define SMI_DG_CASE(N)                                                                          \
    case N:                                                                                     \
      hipLaunchKernelGGL(diag_gauss_rows_kernel<N>, dim3(grid), dim3(kWG), 0, st, a, p0, p1,   \
                         rows, c_ll, c_ent, ll, lik, kl, ent);                                  \
      break;
    switch (A) {
      SMI_DG_CASE(1) SMI_DG_CASE(2) SMI_DG_CASE(3) SMI_DG_CASE(4)
      SMI_DG_CASE(5) SMI_DG_CASE(6) SMI_DG_CASE(7) SMI_DG_CASE(8)
    }
#undef SMI_DG_CASE
    return check_launch("diag_gauss_rows_kernel");
  }
  const size_t lds = (size_t)DG_R * ((A | 1) + 2 * ((2 * A) | 1)) * 4;
  if (lds > 160 * 1024) return set_error(SMI_E_NOFIT, "diag_gauss: act_dim too large");
  allow_lds(diag_gauss_kernel, lds);
  hipLaunchKernelGGL(diag_gauss_kernel, dim3(grid_for(rows, 4096)), dim3(kWG), lds, st, a, p0, p1,
                     rows, A, c_ll, c_ent, ll, lik, kl, ent);
  return check_launch("diag_gauss_kernel");
}

int launch_mlp_forward(const float* params, int in, int h1, int h2, int out, int act, int lv,
                       const float* x, int64_t rows, int64_t stride, int use_zf,
                       const float* zs, const float* zsq, const float* zc, float zeps,
                       float* y, hipStream_t st) {
  MlpFwdArgs a;
  a.params = params; a.in = in; a.h1 = h1; a.h2 = h2; a.out = out; a.act = act; a.lv = lv;
  a.x = x; a.rows = rows; a.stride = stride; a.use_zf = use_zf; a.zsum = zs; a.zsumsq = zsq;
  a.zcount = zc; a.zeps = zeps; a.y = y;
  const MlpLayout L = mlp_layout(in, h1, h2, out, lv);
  const int64_t base = 2 * round4(in) +
                       (int64_t)kRT * (pad_ld(in) + pad_ld(h1) + pad_ld(h2) + pad_small(out));
  a.params_in_lds = ((base + L.pcount) * 4 <= 64 * 1024) ? 1 : 0;
  const int64_t lds = (base + (a.params_in_lds ? L.pcount : 0)) * 4;
  if (lds > 160 * 1024) return set_error(SMI_E_NOFIT, "mlp_forward: LDS does not fit");
  const int64_t ntiles = (rows + kRT - 1) / kRT;
  if (ntiles == 0) return SMI_OK;
  const int grid = (int)(ntiles < 1024 ? ntiles : 1024);
  allow_lds(mlp_forward_kernel, (size_t)lds);
  hipLaunchKernelGGL(mlp_forward_kernel, dim3(grid), dim3(kWG), (size_t)lds, st, a);
  return check_launch("mlp_forward_kernel");
}

int launch_moments(const float* x, int64_t n, const double* part, int np, double* out,
                   hipStream_t st) {
  if ((part && np > 0) || n <= (int64_t)1 << 16) {
    hipLaunchKernelGGL(moments_kernel, dim3(1), dim3(kWG), 0, st, x, n, part, np, out);
    return check_launch("moments_kernel");
  }
  const int grid = grid_for((n + 7) / 8, 1024);
  double* ws = reinterpret_cast<double*>(workspace_f32(4 * grid));
  if (!ws) return set_error(SMI_E_ARG, "moments: workspace unavailable");
  hipLaunchKernelGGL(moments_partial_kernel, dim3(grid), dim3(kWG), 0, st, x, n, ws);
  int rc = check_launch("moments_partial_kernel");
  if (rc) return rc;
  hipLaunchKernelGGL(moments_kernel, dim3(1), dim3(kWG), 0, st, nullptr, n, ws, grid, out);
  return check_launch("moments_kernel");
}

int launch_adam_clip(float* p, const float* g, float* m, float* v, int64_t n, int* step,
                     const float* lr, float b1, float b2, float eps, float wd, float max_norm,
                     float clip_value, const int* skip, float* norm_out, hipStream_t st) {
  static const int gcap = [] { const char* e = getenv("SMI_ADAM_GRID"); return e ? atoi(e) : 2048; }();
  const int grid = grid_for((n + 3) / 4, gcap > 0 && gcap <= 2048 ? gcap : 2048);
  const bool need_norm = max_norm > 0.f || norm_out != nullptr;
  double* part = nullptr;
  if (need_norm) {
    part = reinterpret_cast<double*>(workspace_f32(2 * 2048));
    if (!part) return set_error(SMI_E_ARG, "adam: workspace unavailable");
    hipLaunchKernelGGL(sumsq_partial_kernel, dim3(grid), dim3(kWG), 0, st, g, n, clip_value, part);
    const int rc0 = check_launch("sumsq_partial_kernel");
    if (rc0) return rc0;
  }
  // nontemporal loads and stores of p, g, m, v from SMI_ADAM_NT_MIN (2^24)
  // parameters: streams read and written once per launch, past the caches.
  // Measured (67 M parameters, tools/bench_hbm.py, one MI355X): plain 0.61 /
  // 0.61 of HBM (clip / no clip), nontemporal stores 0.62 / 0.62, both 0.75 /
  // 0.67.  A/B knob SMI_ADAM_NT: 0 plain, 1 stores, 2 loads, 3 both (default).
  static const int nt_v = [] { const char* e = getenv("SMI_ADAM_NT"); return e ? atoi(e) & 3 : 3; }();
  static const int64_t nt_min = [] {
    const char* e = getenv("SMI_ADAM_NT_MIN"); return e ? (int64_t)atoll(e) : (int64_t)1 << 24; }();
  const int ntv = n >= nt_min ? nt_v : 0;
  auto kfn = ntv == 1 ? adam_kernel<1> : ntv == 2 ? adam_kernel<2> : ntv == 3 ? adam_kernel<3>
                                                                    : adam_kernel<0>;
  hipLaunchKernelGGL(kfn, dim3(grid), dim3(kWG), 0, st, p, g, m, v, n, step, lr, b1, b2,
                     eps, wd, max_norm, clip_value, part, need_norm ? grid : 0, skip, norm_out);
  int rc = check_launch("adam_kernel");
  if (rc) return rc;
  hipLaunchKernelGGL(step_inc_kernel, dim3(1), dim3(1), 0, st, step, skip);
  return check_launch("step_inc_kernel");
}

// data-parallel z_update: add all-reduced column sums into the running buffers
__global__ void __launch_bounds__(kWG)
zfilter_accumulate_kernel(const float* __restrict__ s, const float* __restrict__ s2, int dim,
                          float rows, float* rs, float* rsq, float* cnt) {
  for (int c = threadIdx.x; c < dim; c += kWG) {
    rs[c] += s[c];
    rsq[c] += s2[c];
  }
  if (threadIdx.x == 0) cnt[0] += rows;
}

int launch_zfilter_accumulate(const float* s, const float* s2, int dim, float rows, float* rs,
                              float* rsq, float* cnt, hipStream_t st) {
  hipLaunchKernelGGL(zfilter_accumulate_kernel, dim3(1), dim3(kWG), 0, st, s, s2, dim, rows, rs,
                     rsq, cnt);
  return check_launch("zfilter_accumulate_kernel");
}

int launch_ddpg_target(const float* r, const float* d, const float* q, const float* q2,
                       int64_t n, float gn, float* y, hipStream_t st) {
  hipLaunchKernelGGL(ddpg_target_kernel, dim3(grid_for(n)), dim3(kWG), 0, st, r, d, q, q2, n, gn,
                     y);
  return check_launch("ddpg_target_kernel");
}

}  // namespace smi
