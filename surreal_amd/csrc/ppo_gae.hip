// ppo_gae.hip — PPO learner GAE/returns on gfx950.
//
//   critic_gae_kernel      PPOLearner._gae_and_return, non-RNN (ppo.py:355-418):
//                          critic MLP over cat(obs, obs_next) + window sums
//   gae_windows_kernel     windowed GAE given values (ppo.py:387-406), streaming
//
// Numerics follow the reference's fp32 op order where it is observable
// (see DESIGN.md §Numerics).
#include "smi_device.hpp"
#include "smi_internal.hpp"
namespace smi {

// ============================================================ critic + GAE
// One workgroup loops over chunks of CS whole segments (grid-stride).  The
// chunk's rows (b, t), t in [0, T] (t == T is obs_next) are flattened and run
// through the critic MLP in 64-row tiles; values stay in LDS, then one thread
// per segment forms the window sums.
struct CriticGaeArgs {
  const float* params; int D, H1, H2;
  int use_zf; const float *zf_sum, *zf_sumsq, *zf_count; float zf_eps;
  const float *obs, *obs_next, *rewards, *dones;
  int B, T, CS;
  const float *gtab, *ltab; float gamma, gamma_T;
  float *values, *adv, *ret;
  int params_in_lds;
};

__global__ void __launch_bounds__(kWG)
critic_gae_kernel(CriticGaeArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const MlpLayout L = mlp_layout(a.D, a.H1, a.H2, 1, 0);
  const int ldX = pad_ld(a.D), ldH1 = pad_ld(a.H1), ldH2 = pad_ld(a.H2), ldO = pad_small(1);
  const int T1 = a.T + 1;
  // LDS carve (floats)
  float* zmean = sm;                       // [D]
  float* zstd = zmean + round4(a.D);       // [D]
  float* X0 = zstd + round4(a.D);          // [64][ldX]
  float* H1 = X0 + kRT * ldX;              // [64][ldH1]
  float* H2 = H1 + kRT * ldH1;             // [64][ldH2]
  float* OUT = H2 + kRT * ldH2;            // [64][ldO]
  float* vals = OUT + kRT * ldO;           // [CS*T1]
  float* P = vals + round4(a.CS * T1);     // padded params (if in LDS)

  if (a.use_zf) zfilter_colstats(a.zf_sum, a.zf_sumsq, a.zf_count, a.zf_eps, a.D, zmean, zstd);
  MlpView V;
  if (a.params_in_lds) {
    mlp_load_lds(L, a.params, P);
    V = view_padded(L, P);
  } else {
    V = view_flat(L, a.params);
  }
  // zero H/OUT padding columns once (finite values only are ever written)
  for (int e = threadIdx.x; e < kRT * (ldH1 + ldH2 + ldO); e += kWG) H1[e] = 0.f;
  __syncthreads();

  const int nchunks = (a.B + a.CS - 1) / a.CS;
  for (int ch = blockIdx.x; ch < nchunks; ch += gridDim.x) {
    const int b0 = ch * a.CS;
    const int nseg = min(a.CS, a.B - b0);
    const int rows = nseg * T1;
    for (int r0 = 0; r0 < rows; r0 += kRT) {
      // gather rows (b, t) -> X0 with the ZFilter fused
      for (int e = threadIdx.x; e < kRT * ldX; e += kWG) {
        const int r = e / ldX, c = e - r * ldX;
        const int q = r0 + r;
        float v = 0.f;
        if (q < rows && c < a.D) {
          const int sb = q / T1, t = q - sb * T1;
          const int64_t b = b0 + sb;
          v = (t < a.T) ? a.obs[(b * a.T + t) * a.D + c] : a.obs_next[b * a.D + c];
          if (a.use_zf) {
            v = (v - zmean[c]) / zstd[c];
            v = fminf(fmaxf(v, -5.f), 5.f);
          }
        }
        X0[e] = v;
      }
      __syncthreads();
      dense_fwd<ACT_RELU>(X0, ldX, V.W1, V.ld1, V.b1, a.D, a.H1, H1, ldH1);
      __syncthreads();
      dense_fwd<ACT_RELU>(H1, ldH1, V.W2, V.ld2, V.b2, a.H1, a.H2, H2, ldH2);
      __syncthreads();
      dense_fwd<ACT_NONE>(H2, ldH2, V.W3, V.ld3, V.b3, a.H2, 1, OUT, ldO);
      __syncthreads();
      for (int r = threadIdx.x; r < kRT; r += kWG)
        if (r0 + r < rows) vals[r0 + r] = OUT[r * ldO];
      __syncthreads();
    }
    // values[:, 1:] *= 1 - dones   (ppo.py:387)
    for (int q = threadIdx.x; q < rows; q += kWG) {
      const int sb = q / T1, t = q - sb * T1;
      if (t > 0) {
        const int64_t b = b0 + sb;
        vals[q] = vals[q] * (1.f - a.dones[b * a.T + t - 1]);
      }
      if (a.values) a.values[(int64_t)b0 * T1 + q] = vals[q];
    }
    __syncthreads();
    // window sums (ppo.py:409-411), one thread per segment
    for (int sb = threadIdx.x; sb < nseg; sb += kWG) {
      const int64_t b = b0 + sb;
      const float* r = a.rewards + b * a.T;
      const float* v = vals + sb * T1;
      float sr = 0.f, sa = 0.f;
      for (int t = 0; t < a.T; ++t) {
        sr += a.gtab[t] * r[t];
        const float td = (r[t] + a.gamma * v[t + 1]) - v[t];
        sa += (td * a.gtab[t]) * a.ltab[t];
      }
      a.ret[b] = sr + v[a.T] * a.gamma_T;
      a.adv[b] = sa;
    }
    __syncthreads();
  }
}

// ===================================================== streaming GAE windows
// values [B][T+1] (masked in place), rewards/dones [B][T] -> adv/ret [B][E].
// A workgroup stages a contiguous block of SB segments of r, d, V through LDS
// with coalesced loads (the three arrays are contiguous per segment block),
// computes the windows from LDS and writes adv/ret coalesced.
struct GaeWinArgs {
  float* values; const float *rewards, *dones;
  int64_t B; int T, H, E, SB;
  const float *gtab, *ltab; float gamma, gamma_H;
  float *adv, *ret; double* partials;
};

__global__ void __launch_bounds__(kWG)
gae_windows_kernel(GaeWinArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  __shared__ double red[kNW];
  const int T = a.T, T1 = T + 1, H = a.H, E = a.E;
  float* sr = sm;                         // [SB*T]
  float* sd = sr + a.SB * T;              // [SB*T]
  float* sv = sd + a.SB * T;              // [SB*T1]
  float* sg = sv + a.SB * T1;             // [H] gamma table
  float* sl = sg + H;                     // [H] lambda table
  for (int k = threadIdx.x; k < H; k += kWG) { sg[k] = a.gtab[k]; sl[k] = a.ltab[k]; }
  double psum = 0.0, psq = 0.0;
  const int64_t nblk = (a.B + a.SB - 1) / a.SB;
  for (int64_t blk = blockIdx.x; blk < nblk; blk += gridDim.x) {
    const int64_t b0 = blk * a.SB;
    const int nseg = (int)min((int64_t)a.SB, a.B - b0);
    const int nrd = nseg * T, nv = nseg * T1;
    const float* gr = a.rewards + b0 * T;
    const float* gd = a.dones + b0 * T;
    float* gv = a.values + b0 * T1;
    __syncthreads();
    for (int i = threadIdx.x; i < nrd; i += kWG) { sr[i] = gr[i]; sd[i] = gd[i]; }
    for (int i = threadIdx.x; i < nv; i += kWG) sv[i] = gv[i];
    __syncthreads();
    // mask values[:,1:] *= 1-dones and write back
    for (int i = threadIdx.x; i < nv; i += kWG) {
      const int s = i / T1, t = i - s * T1;
      if (t > 0) {
        const float m = sv[i] * (1.f - sd[s * T + t - 1]);
        sv[i] = m;
        gv[i] = m;
      }
    }
    __syncthreads();
    // windows: item = (segment s, window w)
    const int nitems = nseg * E;
    for (int it = threadIdx.x; it < nitems; it += kWG) {
      const int s = it / E, w = it - s * E;
      const float* r = sr + s * T + w;
      const float* v = sv + s * T1 + w;
      float rs = 0.f, as = 0.f;
      for (int k = 0; k < H; ++k) {
        rs += sg[k] * r[k];
        const float td = (r[k] + a.gamma * v[k + 1]) - v[k];
        as += (td * sg[k]) * sl[k];
      }
      const int64_t o = (b0 + s) * E + w;
      a.ret[o] = rs + v[H] * a.gamma_H;
      a.adv[o] = as;
      psum += (double)as;
      psq += (double)as * (double)as;
    }
  }
  const double s1 = block_sum_d(psum, red);
  const double s2 = block_sum_d(psq, red);
  if (threadIdx.x == 0 && a.partials) {
    a.partials[2 * blockIdx.x] = s1;
    a.partials[2 * blockIdx.x + 1] = s2;
  }
}

// ============================================================ host launchers
int launch_critic_gae(const float* critic_params, int D, int H1, int H2, int use_zf,
                      const float* zf_sum, const float* zf_sumsq, const float* zf_count,
                      float zf_eps, const float* obs, const float* obs_next,
                      const float* rewards, const float* dones, int B, int T,
                      const float* gtab, const float* ltab, float gamma, float gamma_T,
                      float* values, float* adv, float* ret, hipStream_t stream) {
  CriticGaeArgs a;
  a.params = critic_params; a.D = D; a.H1 = H1; a.H2 = H2;
  a.use_zf = use_zf; a.zf_sum = zf_sum; a.zf_sumsq = zf_sumsq; a.zf_count = zf_count;
  a.zf_eps = zf_eps;
  a.obs = obs; a.obs_next = obs_next; a.rewards = rewards; a.dones = dones;
  a.B = B; a.T = T;
  a.gtab = gtab; a.ltab = ltab; a.gamma = gamma; a.gamma_T = gamma_T;
  a.values = values; a.adv = adv; a.ret = ret;
  const int T1 = T + 1;
  // segments per chunk: values of a chunk stay in LDS (<= 4096 floats); aim
  // for >= 256 workgroups when the batch is large.
  int CS = 4096 / T1;
  if (CS < 1) CS = 1;
  const int64_t rows_total = (int64_t)B * T1;
  const int want_cs = (int)((rows_total + 256 * kRT - 1) / (256 * kRT) / T1) + 1;
  if (want_cs < CS) CS = want_cs;
  if (CS > B) CS = B;
  a.CS = CS;
  const MlpLayout L = mlp_layout(D, H1, H2, 1, 0);
  const int ldX = pad_ld(D), ldH1 = pad_ld(H1), ldH2 = pad_ld(H2), ldO = pad_small(1);
  int64_t base = 2 * round4(D) + kRT * (ldX + ldH1 + ldH2 + ldO) + round4(CS * T1);
  int64_t with_p = base + L.pcount;
  a.params_in_lds = (with_p * 4 <= 160 * 1024) ? 1 : 0;
  const int64_t lds = (a.params_in_lds ? with_p : base) * 4;
  if (lds > 160 * 1024) return set_error(SMI_E_NOFIT, "critic_gae: LDS does not fit");
  const int nchunks = (B + CS - 1) / CS;
  const int grid = nchunks < 2048 ? nchunks : 2048;
  allow_lds(critic_gae_kernel, (size_t)lds);
  hipLaunchKernelGGL(critic_gae_kernel, dim3(grid), dim3(kWG), (size_t)lds, stream, a);
  return check_launch("critic_gae_kernel");
}

int gae_windows_max_partials(int64_t B, int T) {
  (void)T;
  (void)B;
  return 2048;
}

int launch_gae_windows(float* values, const float* rewards, const float* dones, int64_t B,
                       int T, int H, const float* gtab, const float* ltab, float gamma,
                       float gamma_H, float* adv, float* ret, double* partials,
                       int* n_partials, hipStream_t stream) {
  if (H < 1 || H > T) return set_error(SMI_E_ARG, "gae_windows: horizon must be in [1, T]");
  GaeWinArgs a;
  a.values = values; a.rewards = rewards; a.dones = dones; a.B = B; a.T = T; a.H = H;
  a.E = T - H + 1;
  // segment block: ~16 KB of r/d/V per block
  int SB = 4096 / (3 * T + 1);
  if (SB < 1) SB = 1;
  a.SB = SB;
  a.gtab = gtab; a.ltab = ltab; a.gamma = gamma; a.gamma_H = gamma_H;
  a.adv = adv; a.ret = ret; a.partials = partials;
  const int64_t nblk = (B + SB - 1) / SB;
  const int grid = (int)(nblk < 2048 ? nblk : 2048);
  const size_t lds = (size_t)(SB * (3 * T + 1) + 2 * H) * 4;
  if (lds > 160 * 1024) return set_error(SMI_E_NOFIT, "gae_windows: T too large");
  allow_lds(gae_windows_kernel, lds);
  hipLaunchKernelGGL(gae_windows_kernel, dim3(grid), dim3(kWG), lds, stream, a);
  if (n_partials) *n_partials = grid;
  return check_launch("gae_windows_kernel");
}

}  // namespace smi
