// ppo_kernels.hip — PPO learner hot path on gfx950.
//
//   critic_gae_kernel      PPOLearner._gae_and_return, non-RNN (ppo.py:355-418)
//   gae_windows_kernel     windowed GAE given values (ppo.py:387-406), streaming
//   ppo_fused_kernel       PPOLearner._optimize epochs (ppo.py:487-586), one CU
//                          per loop: WG0 policy epochs, WG1 value epochs
//
// Numerics follow the reference's fp32 op order where it is observable
// (see DESIGN.md §Numerics); reductions that the reference does with torch's
// double-accumulated CPU kernels (std/var) are done in fp64 here.
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

// ============================================================ fused PPO
// LDS layout shared by host (size query) and device.
struct FusedLayout {
  MlpLayout A, C;
  int Bp, ntiles;
  int ldX, ldH1, ldH, ldO, ldDG, ldOc;
  // policy workgroup (float offsets)
  int pP, pG, pX0, pH1, pH2, pOUT, pDG1, pDG2;
  int pRefMu, pMu, pAct, pBeh, pAdv, pBp, pZm, pZs, pRZm, pRZs, pCol, pGS, pScr, pTotal;
  // value workgroup
  int vP, vG, vX0, vH1, vH2, vOUT, vDG1, vDG2, vRet, vV, vZm, vZs, vScr, vTotal;
};

__host__ __device__ inline FusedLayout fused_layout(int B, int D, int H1, int H2, int A,
                                                    int cH1, int cH2) {
  FusedLayout F;
  F.A = mlp_layout(D, H1, H2, A, 1);
  F.C = mlp_layout(D, cH1, cH2, 1, 0);
  F.ntiles = (B + kRT - 1) / kRT;
  F.Bp = F.ntiles * kRT;
  F.ldX = pad_ld(D);
  // policy
  F.ldH1 = pad_ld(H1);
  F.ldH = pad_ld(H1 > H2 ? H1 : H2);
  F.ldO = pad_small(A);
  F.ldDG = F.ldH;
  int o = 0;
  F.pScr = o; o += 32;                        // 16 doubles of reduction scratch
  F.pP = o; o += F.A.pcount;
  F.pG = o; o += F.A.pcount;
  F.pX0 = o; o += kRT * F.ldX;
  F.pH1 = o; o += kRT * F.ldH1;
  F.pH2 = o; o += kRT * F.ldH;
  F.pOUT = o; o += kRT * F.ldO;
  F.pDG1 = o; o += kRT * F.ldDG;
  F.pDG2 = o; o += kRT * F.ldO;
  F.pRefMu = o; o += round4(F.Bp * A);
  F.pMu = o; o += round4(F.Bp * A);
  F.pAct = o; o += round4(F.Bp * A);
  F.pBeh = o; o += round4(F.Bp * 2 * A);
  F.pAdv = o; o += F.Bp;
  F.pBp = o; o += F.Bp;
  F.pZm = o; o += round4(D);
  F.pZs = o; o += round4(D);
  F.pRZm = o; o += round4(D);
  F.pRZs = o; o += round4(D);
  F.pCol = o; o += round4(6 * A);             // sig, logsig, refsig, reflogsig, gsig, spare
  F.pGS = o; o += round4(kRT * A);            // per-row d loss / d sigma of a tile
  F.pTotal = o;
  // value
  const int ldCH1 = pad_ld(cH1), ldCH = pad_ld(cH1 > cH2 ? cH1 : cH2);
  F.ldOc = pad_small(1);
  o = 0;
  F.vScr = o; o += 32;
  F.vP = o; o += F.C.pcount;
  F.vG = o; o += F.C.pcount;
  F.vX0 = o; o += kRT * F.ldX;
  F.vH1 = o; o += kRT * ldCH1;
  F.vH2 = o; o += kRT * ldCH;
  F.vOUT = o; o += kRT * F.ldOc;
  F.vDG1 = o; o += kRT * ldCH;
  F.vDG2 = o; o += kRT * F.ldOc;
  F.vRet = o; o += F.Bp;
  F.vV = o; o += F.Bp;
  F.vZm = o; o += round4(D);
  F.vZs = o; o += round4(D);
  F.vTotal = o;
  return F;
}

int64_t fused_lds_bytes(int B, int D, int H1, int H2, int A, int cH1, int cH2) {
  const FusedLayout F = fused_layout(B, D, H1, H2, A, cH1, cH2);
  const int64_t f = F.pTotal > F.vTotal ? F.pTotal : F.vTotal;
  return f * 4;
}

// --- DiagGauss row helpers (ppo_net.py:29-72), one thread per row ---------
__device__ inline float dg_loglik(const float* act, const float* mu, const float* sd,
                                  const float* logsd, int A, float c_loglik) {
  float s = 0.f, l = 0.f;
  for (int j = 0; j < A; ++j) {
    const float u = (act[j] - mu[j]) / sd[j];
    s += u * u;
    l += logsd[j];
  }
  return (-0.5f * s - c_loglik) - l;
}
// same, with a per-element log of the row's own std (behaviour policy rows)
__device__ inline float dg_loglik_rowstd(const float* act, const float* mu, const float* sd,
                                         int A, float c_loglik) {
  float s = 0.f, l = 0.f;
  for (int j = 0; j < A; ++j) {
    const float u = (act[j] - mu[j]) / sd[j];
    s += u * u;
    l += logf(sd[j]);
  }
  return (-0.5f * s - c_loglik) - l;
}
// KL(p0 || p1) with p0 = (mu0, sd0), p1 = (mu1, sd1)
__device__ inline float dg_kl(const float* mu0, const float* sd0, const float* mu1,
                              const float* sd1, int A) {
  float s1 = 0.f, s2 = 0.f;
  for (int j = 0; j < A; ++j) {
    s1 += logf(sd1[j] / sd0[j]);
    const float d = mu0[j] - mu1[j];
    s2 += (sd0[j] * sd0[j] + d * d) / (2.f * (sd1[j] * sd1[j]));
  }
  return (s1 + s2) - 0.5f * (float)A;
}

struct FusedCtx {
  const smi_ppo_args* a;
  FusedLayout F;
  float* sm;
  float c_loglik;   // 0.5*log(2pi)*A  (rounded from double, as torch does)
  float c_entropy;  // 0.5*log(2pi e)*A
};

// actor forward of one 64-row tile into the policy buffers
__device__ void policy_fwd_tile(const FusedCtx& c, const MlpView& V, int tile,
                                const float* zm, const float* zs) {
  const smi_ppo_args& a = *c.a;
  const FusedLayout& F = c.F;
  float* sm = c.sm;
  const int r0 = tile * kRT;
  const int nr = min(kRT, a.B - r0);
  load_obs_tile(a.obs + (int64_t)r0 * a.obs_stride, a.obs_stride, nr, a.obs_dim,
                a.use_zf ? zm : nullptr, zs, sm + F.pX0, F.ldX);
  __syncthreads();
  dense_fwd<ACT_RELU>(sm + F.pX0, F.ldX, V.W1, V.ld1, V.b1, a.obs_dim, a.h1, sm + F.pH1, F.ldH1);
  __syncthreads();
  dense_fwd<ACT_RELU>(sm + F.pH1, F.ldH1, V.W2, V.ld2, V.b2, a.h1, a.h2, sm + F.pH2, F.ldH);
  __syncthreads();
  dense_fwd<ACT_TANH>(sm + F.pH2, F.ldH, V.W3, V.ld3, V.b3, a.h2, a.act_dim, sm + F.pOUT, F.ldO);
  __syncthreads();
}

// Adam on a padded LDS parameter image (torch.optim.Adam single-tensor path,
// torch/optim/adam.py): m.lerp_(g, 1-b1); v.mul_(b2).addcmul_(g, g, 1-b2);
// p.addcdiv_(m, v.sqrt()/sqrt(bc2) + eps, value=-lr/bc1).
__device__ void adam_lds(const MlpLayout& L, float* P, const float* G, float* m, float* v,
                         int t, float lr, float beta1, float beta2, float eps,
                         float wd, float coef) {
  __syncthreads();
  const double bc1 = 1.0 - pow((double)beta1, (double)t);
  const double bc2 = 1.0 - pow((double)beta2, (double)t);
  const float step_size = (float)((double)lr / bc1);
  const float bc2_sqrt = (float)sqrt(bc2);
  const float w1 = (float)(1.0 - (double)beta1);
  const float w2 = (float)(1.0 - (double)beta2);
  for (int i = threadIdx.x; i < L.fcount; i += kWG) {
    const int pi = mlp_flat_to_pad(L, i);
    float g = G[pi] * coef;
    float p = P[pi];
    if (wd != 0.f) g = g + wd * p;
    float mi = m[i], vi = v[i];
    mi = mi + w1 * (g - mi);
    vi = vi * beta2 + (w2 * g) * g;
    const float denom = sqrtf(vi) / bc2_sqrt + eps;
    p = p + (-step_size) * (mi / denom);
    m[i] = mi; v[i] = vi; P[pi] = p;
  }
  __syncthreads();
}

// global L2 norm of the (unpadded) gradient, fp64 accumulation
__device__ float grad_norm_lds(const MlpLayout& L, const float* G, double* scr) {
  double s = 0.0;
  for (int i = threadIdx.x; i < L.fcount; i += kWG) {
    const float g = G[mlp_flat_to_pad(L, i)];
    s += (double)g * (double)g;
  }
  s = block_sum_d(s, scr);
  return (float)sqrt(s);
}

__device__ void policy_wg(const FusedCtx& c) {
  const smi_ppo_args& a = *c.a;
  const FusedLayout& F = c.F;
  float* sm = c.sm;
  double* scr = reinterpret_cast<double*>(sm + F.pScr);
  const int A = a.act_dim, B = a.B;
  float* P = sm + F.pP;
  float* G = sm + F.pG;
  float* refmu = sm + F.pRefMu;
  float* mu = sm + F.pMu;
  float* act = sm + F.pAct;
  float* beh = sm + F.pBeh;
  float* adv = sm + F.pAdv;
  float* bpl = sm + F.pBp;
  float* zm = sm + F.pZm; float* zs = sm + F.pZs;
  float* rzm = sm + F.pRZm; float* rzs = sm + F.pRZs;
  float* sig = sm + F.pCol;
  float* logsig = sig + A;
  float* refsig = logsig + A;
  float* reflogsig = refsig + A;
  float* gsig = reflogsig + A;
  const float clip_lo = a.hyper[SMI_HYPX_CLIP_LO];
  const float clip_hi = a.hyper[SMI_HYPX_CLIP_HI];
  const float beta = a.hyper[SMI_HYP_BETA];
  const float lr = a.hyper[SMI_HYP_LR_ACTOR];
  const float invB = 1.f / (float)B;

  // zero all activation buffers (keeps padding columns finite)
  for (int e = F.pX0 + threadIdx.x; e < F.pRefMu; e += kWG) sm[e] = 0.f;
  if (a.use_zf) {
    zfilter_colstats(a.zf_sum, a.zf_sumsq, a.zf_count, a.zf_eps, a.obs_dim, zm, zs);
    zfilter_colstats(a.rzf_sum, a.rzf_sumsq, a.rzf_count, a.zf_eps, a.obs_dim, rzm, rzs);
  }
  // per-row inputs
  for (int e = threadIdx.x; e < F.Bp * A; e += kWG) {
    const int r = e / A, j = e - r * A;
    act[e] = r < B ? a.actions[(int64_t)r * a.act_stride + j] : 0.f;
    beh[r * 2 * A + j] = r < B ? a.behave[(int64_t)r * a.beh_stride + j] : 0.f;
    beh[r * 2 * A + A + j] = r < B ? a.behave[(int64_t)r * a.beh_stride + A + j] : 1.f;
  }
  // advantage normalisation (ppo.py:413-416): unbiased std, max(std, 1e-4)
  {
    double s1, s2, n;
    if (a.adv_moments) {
      s1 = a.adv_moments[0]; s2 = a.adv_moments[1]; n = a.adv_moments[2];
    } else {
      double l1 = 0.0;
      for (int r = threadIdx.x; r < B; r += kWG) l1 += (double)a.adv_raw[r];
      s1 = block_sum_d(l1, scr);
      n = (double)B;
      const double mean = s1 / n;
      double l2 = 0.0;
      for (int r = threadIdx.x; r < B; r += kWG) {
        const double d = (double)a.adv_raw[r] - mean;
        l2 += d * d;
      }
      s2 = block_sum_d(l2, scr) + n * mean * mean;   // back to a raw sum of squares
    }
    const double mean_d = s1 / n;
    const double var_d = (s2 - n * mean_d * mean_d) / (n - 1.0);
    const float mean_f = (float)mean_d;
    float std_f = (float)sqrt(var_d > 0.0 ? var_d : 0.0);
    const float denom = std_f > 1e-4f ? std_f : 1e-4f;
    for (int r = threadIdx.x; r < F.Bp; r += kWG) {
      float v = 0.f;
      if (r < B) v = a.norm_adv ? (a.adv_raw[r] - mean_f) / denom : a.adv_raw[r];
      adv[r] = v;
    }
  }
  __syncthreads();
  // behaviour likelihood per row (reused by every epoch)
  for (int r = threadIdx.x; r < F.Bp; r += kWG) {
    float v = 1.f;
    if (r < B) {
      const float* p = beh + r * 2 * A;
      const float ll = dg_loglik_rowstd(act + r * A, p, p + A, A, c.c_loglik);
      v = fmaxf(expf(ll), 1e-5f);
    }
    bpl[r] = v;
  }
  // ---- reference policy: ref_target_model.forward_actor(obs_iter) (ppo.py:539)
  mlp_load_lds(F.A, a.ref_actor, P);
  {
    const MlpView V = view_padded(F.A, P);
    for (int j = threadIdx.x; j < A; j += kWG) {
      refsig[j] = expf(V.lv[j]);
      reflogsig[j] = logf(refsig[j]);
    }
    for (int tile = 0; tile < F.ntiles; ++tile) {
      policy_fwd_tile(c, V, tile, rzm, rzs);
      for (int e = threadIdx.x; e < kRT * A; e += kWG) {
        const int r = e / A, j = e - r * A;
        refmu[(tile * kRT + r) * A + j] = sm[F.pOUT + r * F.ldO + j];
      }
      __syncthreads();
    }
  }
  // ---- model actor into LDS
  mlp_load_lds(F.A, a.actor, P);
  for (int i = threadIdx.x; i < F.A.pcount; i += kWG) G[i] = 0.f;
  const MlpView V = view_padded(F.A, P);
  __syncthreads();

  float st_surr = 0.f, st_clip = 0.f, st_kladapt = 0.f, st_ent = 0.f, st_gnorm = 0.f;
  float st_klad = 0.f, pol_kl = 0.f;
  int epochs_run = 0;
  int astep = a.actor_step[0];
  const int E = a.epoch_policy;
  for (int e = 0; e <= E; ++e) {
    // sigma = exp(log_var) broadcast (builders.py:127)
    for (int j = threadIdx.x; j < A; j += kWG) {
      sig[j] = expf(V.lv[j]);
      logsig[j] = logf(sig[j]);
    }
    __syncthreads();
    // forward all tiles; KL(ref || current) per row
    float klp = 0.f;
    for (int tile = 0; tile < F.ntiles; ++tile) {
      policy_fwd_tile(c, V, tile, zm, zs);
      for (int ee = threadIdx.x; ee < kRT * A; ee += kWG) {
        const int r = ee / A, j = ee - r * A;
        mu[(tile * kRT + r) * A + j] = sm[F.pOUT + r * F.ldO + j];
      }
      __syncthreads();
      for (int r = threadIdx.x; r < kRT; r += kWG) {
        const int gr = tile * kRT + r;
        if (gr < B) klp += dg_kl(refmu + gr * A, refsig, mu + gr * A, sig, A);
      }
    }
    const float kl = block_sum_f(klp, scr) * invB;
    if (e > 0) {
      pol_kl = kl;                                  // ppo.py:553-555
      if ((double)kl > a.kl_target * 4.0) break;   // ppo.py:556-557 (python float compare)
    }
    if (e == E) break;
    // ---- loss + backward (one pass per tile; single tile keeps activations)
    float coef_kl = 0.f;
    if (a.mode == 1) {
      coef_kl = beta;
      if ((double)kl - 2.0 * (double)a.kl_target > 0.0)      // ppo.py:275-276
        coef_kl = beta + a.kl_cutoff_coeff * 2.f * (kl - (float)(2.0 * a.kl_target));
    }
    for (int j = threadIdx.x; j < A; j += kWG) gsig[j] = 0.f;
    float p_surr = 0.f, p_clip = 0.f;
    for (int tile = 0; tile < F.ntiles; ++tile) {
      if (F.ntiles > 1) policy_fwd_tile(c, V, tile, zm, zs);
      float* dOut = sm + F.pDG2;
      float* gsr = sm + F.pGS;
      for (int r = threadIdx.x; r < kRT; r += kWG) {
        const int gr = tile * kRT + r;
        float* dz = dOut + r * F.ldO;
        if (gr >= B) {
          for (int j = 0; j < F.ldO; ++j) dz[j] = 0.f;
          for (int j = 0; j < A; ++j) gsr[r * A + j] = 0.f;
          continue;
        }
        const float* m = mu + gr * A;
        const float* ac = act + gr * A;
        const float ll = dg_loglik(ac, m, sig, logsig, A, c.c_loglik);
        const float ex = expf(ll);
        const float lp = fmaxf(ex, 1e-5f);
        const float bp = bpl[gr];
        const float av = adv[gr];
        float g_lp;
        if (a.mode == 0) {
          // clip loss (ppo.py:209-217)
          const float ratio = lp / bp;
          const float cr = fminf(fmaxf(ratio, clip_lo), clip_hi);
          const float surr = -ratio * av;
          const float csur = -cr * av;
          p_surr += surr;
          p_clip += fmaxf(surr, csur);
          const float g_ratio = (surr >= csur) ? -(invB * av) : 0.f;
          g_lp = g_ratio / bp;
        } else {
          // adapt surrogate (ppo.py:267-272)
          const float bpc = fmaxf(bp, 1e-2f);
          p_surr += av * (lp / bpc);
          g_lp = (-invB * av) / bpc;
        }
        const float g_ll = (ex >= 1e-5f) ? g_lp * ex : 0.f;
        const float gkl = coef_kl * invB;
        for (int j = 0; j < A; ++j) {
          const float u = (ac[j] - m[j]) / sig[j];
          float gmu = g_ll * (u / sig[j]);
          float gsd = g_ll * (u * u / sig[j] - 1.f / sig[j]);
          if (a.mode == 1) {
            const float d = refmu[gr * A + j] - m[j];
            const float s1 = sig[j];
            gmu += gkl * (-d / (s1 * s1));
            gsd += gkl * (1.f / s1 - (refsig[j] * refsig[j] + d * d) / (s1 * s1 * s1));
          }
          gsr[r * A + j] = gsd;
          dz[j] = gmu * (1.f - m[j] * m[j]);     // tanh backward
        }
        for (int j = A; j < F.ldO; ++j) dz[j] = 0.f;
      }
      __syncthreads();
      for (int j = threadIdx.x; j < A; j += kWG) {
        float s = 0.f;
        for (int r = 0; r < kRT; ++r) s += gsr[r * A + j];
        gsig[j] += s;
      }
      __syncthreads();
      // backward through the MLP (accumulates into G)
      float* X0 = sm + F.pX0; float* H1 = sm + F.pH1; float* H2 = sm + F.pH2;
      float* DG1 = sm + F.pDG1;
      const MlpLayout& L = F.A;
      dense_bwd_dw(dOut, F.ldO, H2, F.ldH, a.h2, A, G + L.pW3, L.ld3, G + L.pb3);
      dense_bwd_dx<ACT_RELU>(dOut, F.ldO, V.W3, V.ld3, a.h2, A, H2, F.ldH, DG1, F.ldDG);
      __syncthreads();
      dense_bwd_dw(DG1, F.ldDG, H1, F.ldH1, a.h1, a.h2, G + L.pW2, L.ld2, G + L.pb2);
      dense_bwd_dx<ACT_RELU>(DG1, F.ldDG, V.W2, V.ld2, a.h1, a.h2, H1, F.ldH1, H2, F.ldH);
      __syncthreads();
      dense_bwd_dw(H2, F.ldH, X0, F.ldX, a.obs_dim, a.h1, G + L.pW1, L.ld1, G + L.pb1);
      __syncthreads();
    }
    // log_var gradient: sigma = exp(log_var) * ones  ->  sum_rows g_sigma * sigma
    for (int j = threadIdx.x; j < A; j += kWG) G[F.A.plv + j] = gsig[j] * sig[j];
    __syncthreads();
    // stats of this update
    const float tot_surr = block_sum_f(p_surr, scr);
    const float tot_clip = block_sum_f(p_clip, scr);
    float ent = 0.f;
    for (int j = 0; j < A; ++j) ent += logsig[j];
    ent = 0.5f * ent + c.c_entropy;
    if (a.mode == 0) {
      st_surr = tot_surr * invB;
      st_clip = tot_clip * invB;
    } else {
      const float surr = -(tot_surr * invB);
      float loss = surr + beta * kl;
      if ((double)kl - 2.0 * (double)a.kl_target > 0.0) {
        const float d = kl - (float)(2.0 * a.kl_target);
        loss = loss + a.kl_cutoff_coeff * (d * d);
      }
      st_surr = surr;
      st_kladapt = loss;
      st_klad = kl;
    }
    st_ent = ent;
    // clip_grad_norm_ (ppo.py:243-246) + Adam (ppo.py:247)
    const float norm = grad_norm_lds(F.A, G, scr);
    float coef = 1.f;
    if (a.clip_actor_grad) {
      const float cc = a.actor_max_norm / (norm + 1e-6f);
      coef = cc < 1.f ? cc : 1.f;
      st_gnorm = norm;
    }
    ++astep;
    adam_lds(F.A, P, G, a.actor_m, a.actor_v, astep, lr, a.beta1, a.beta2,
             a.adam_eps, a.actor_wd, coef);
    for (int i = threadIdx.x; i < F.A.pcount; i += kWG) G[i] = 0.f;
    ++epochs_run;
    __syncthreads();
  }
  // ---- statistics after the loop (ppo.py:559,568-576); mu holds curr_pol
  float p_bl = 0.f, p_isw = 0.f, p_rbd = 0.f;
  for (int r = threadIdx.x; r < B; r += kWG) {
    const float bl = bpl[r];
    const float cl = fmaxf(expf(dg_loglik(act + r * A, mu + r * A, sig, logsig, A, c.c_loglik)), 1e-5f);
    p_bl += bl;
    p_isw += cl / (bl + 1e-4f);
    const float* p = beh + r * 2 * A;
    p_rbd += dg_kl(refmu + r * A, refsig, p, p + A, A);
  }
  const float t_bl = block_sum_f(p_bl, scr);
  const float t_isw = block_sum_f(p_isw, scr);
  const float t_rbd = block_sum_f(p_rbd, scr);
  float p_ret = 0.f;
  for (int r = threadIdx.x; r < B; r += kWG) p_ret += a.ret[r];
  const float t_ret = block_sum_f(p_ret, scr);
  mlp_store_flat(F.A, P, a.actor);
  if (threadIdx.x == 0) {
    float lvs = 0.f;
    for (int j = 0; j < A; ++j) lvs += V.lv[j];
    float* st = a.stats;
    st[SMI_ST_SURR_LOSS] = st_surr;
    st[SMI_ST_CLIP_SURR_LOSS] = st_clip;
    st[SMI_ST_KL_LOSS_ADAPT] = st_kladapt;
    st[SMI_ST_ENTROPY] = st_ent;
    st[SMI_ST_POL_KL] = pol_kl;
    st[SMI_ST_GRAD_NORM_ACTOR] = st_gnorm;
    st[SMI_ST_AVG_RETURN] = t_ret * invB;
    st[SMI_ST_AVG_LOG_SIG] = lvs / (float)A;
    st[SMI_ST_AVG_BEHAVE_LIK] = t_bl * invB;
    st[SMI_ST_AVG_IS_WEIGHT] = t_isw * invB;
    st[SMI_ST_REF_BEHAVE_DIFF] = t_rbd * invB;
    st[SMI_ST_EPOCHS_RUN] = (float)epochs_run;
    st[SMI_ST_POL_KL_ADAPT] = st_klad;
    a.actor_step[0] = astep;
    if (a.kl_record && a.kl_count) {
      const int k = a.kl_count[0];
      if (k < a.kl_capacity) a.kl_record[k] = pol_kl;
      a.kl_count[0] = k + 1;
    }
  }
}

__device__ void value_wg(const FusedCtx& c) {
  const smi_ppo_args& a = *c.a;
  const FusedLayout& F = c.F;
  float* sm = c.sm;
  double* scr = reinterpret_cast<double*>(sm + F.vScr);
  const int B = a.B;
  const MlpLayout& L = F.C;
  float* P = sm + F.vP;
  float* G = sm + F.vG;
  float* X0 = sm + F.vX0; float* H1 = sm + F.vH1; float* H2 = sm + F.vH2;
  float* OUT = sm + F.vOUT; float* DG1 = sm + F.vDG1; float* DG2 = sm + F.vDG2;
  float* ret = sm + F.vRet; float* Vv = sm + F.vV;
  float* zm = sm + F.vZm; float* zs = sm + F.vZs;
  const int ldH1 = pad_ld(a.critic_h1), ldH = pad_ld(a.critic_h1 > a.critic_h2 ? a.critic_h1 : a.critic_h2);
  const int ldO = F.ldOc;
  const float lr = a.hyper[SMI_HYP_LR_CRITIC];
  const float invB = 1.f / (float)B;

  for (int e = F.vX0 + threadIdx.x; e < F.vRet; e += kWG) sm[e] = 0.f;
  if (a.use_zf) zfilter_colstats(a.zf_sum, a.zf_sumsq, a.zf_count, a.zf_eps, a.obs_dim, zm, zs);
  for (int r = threadIdx.x; r < F.Bp; r += kWG) ret[r] = r < B ? a.ret[r] : 0.f;
  mlp_load_lds(L, a.critic, P);
  for (int i = threadIdx.x; i < L.pcount; i += kWG) G[i] = 0.f;
  __syncthreads();
  const MlpView V = view_padded(L, P);
  float st_loss = 0.f, st_ev = 0.f, st_gnorm = 0.f;
  int cstep = a.critic_step[0];
  for (int e = 0; e < a.epoch_baseline; ++e) {
    for (int tile = 0; tile < F.ntiles; ++tile) {
      const int r0 = tile * kRT, nr = min(kRT, B - r0);
      load_obs_tile(a.obs + (int64_t)r0 * a.obs_stride, a.obs_stride, nr, a.obs_dim,
                    a.use_zf ? zm : nullptr, zs, X0, F.ldX);
      __syncthreads();
      dense_fwd<ACT_RELU>(X0, F.ldX, V.W1, V.ld1, V.b1, a.obs_dim, a.critic_h1, H1, ldH1);
      __syncthreads();
      dense_fwd<ACT_RELU>(H1, ldH1, V.W2, V.ld2, V.b2, a.critic_h1, a.critic_h2, H2, ldH);
      __syncthreads();
      dense_fwd<ACT_NONE>(H2, ldH, V.W3, V.ld3, V.b3, a.critic_h2, 1, OUT, ldO);
      __syncthreads();
      // value loss gradient: d/dV mean((V-R)^2) = 2 (V-R) / B   (ppo.py:326)
      for (int r = threadIdx.x; r < kRT; r += kWG) {
        const int gr = r0 + r;
        float g = 0.f;
        if (gr < B) {
          const float v = OUT[r * ldO];
          Vv[gr] = v;
          g = invB * (2.f * (v - ret[gr]));
        }
        DG2[r * ldO] = g;
        for (int j = 1; j < ldO; ++j) DG2[r * ldO + j] = 0.f;
      }
      __syncthreads();
      dense_bwd_dw(DG2, ldO, H2, ldH, a.critic_h2, 1, G + L.pW3, L.ld3, G + L.pb3);
      dense_bwd_dx<ACT_RELU>(DG2, ldO, V.W3, V.ld3, a.critic_h2, 1, H2, ldH, DG1, ldH);
      __syncthreads();
      dense_bwd_dw(DG1, ldH, H1, ldH1, a.critic_h1, a.critic_h2, G + L.pW2, L.ld2, G + L.pb2);
      dense_bwd_dx<ACT_RELU>(DG1, ldH, V.W2, V.ld2, a.critic_h1, a.critic_h2, H1, ldH1, H2, ldH);
      __syncthreads();
      dense_bwd_dw(H2, ldH, X0, F.ldX, a.obs_dim, a.critic_h1, G + L.pW1, L.ld1, G + L.pb1);
      __syncthreads();
    }
    // stats (ppo.py:325-331): loss, explained variance with unbiased variances
    double l_se = 0.0, l_d = 0.0, l_r = 0.0;
    for (int r = threadIdx.x; r < B; r += kWG) {
      const double d = (double)ret[r] - (double)Vv[r];
      l_se += (double)((Vv[r] - ret[r]) * (Vv[r] - ret[r]));
      l_d += d; l_r += (double)ret[r];
    }
    const double t_se = block_sum_d(l_se, scr);
    const double mean_d = block_sum_d(l_d, scr) / B;
    const double mean_r = block_sum_d(l_r, scr) / B;
    double q_d = 0.0, q_r = 0.0;
    for (int r = threadIdx.x; r < B; r += kWG) {
      const double d = (double)ret[r] - (double)Vv[r] - mean_d;
      const double rr = (double)ret[r] - mean_r;
      q_d += d * d; q_r += rr * rr;
    }
    const double var_d = block_sum_d(q_d, scr) / (B - 1);
    const double var_r = block_sum_d(q_r, scr) / (B - 1);
    st_loss = (float)(t_se / B);
    st_ev = 1.f - (float)var_d / (float)var_r;
    const float norm = grad_norm_lds(L, G, scr);
    float coef = 1.f;
    if (a.clip_critic_grad) {
      const float cc = a.critic_max_norm / (norm + 1e-6f);
      coef = cc < 1.f ? cc : 1.f;
      st_gnorm = norm;
    }
    ++cstep;
    adam_lds(L, P, G, a.critic_m, a.critic_v, cstep, lr, a.beta1, a.beta2,
             a.adam_eps, a.critic_wd, coef);
    for (int i = threadIdx.x; i < L.pcount; i += kWG) G[i] = 0.f;
    __syncthreads();
  }
  mlp_store_flat(L, P, a.critic);
  if (threadIdx.x == 0) {
    a.stats[SMI_ST_VAL_LOSS] = st_loss;
    a.stats[SMI_ST_VAL_EXPL_VAR] = st_ev;
    a.stats[SMI_ST_GRAD_NORM_CRITIC] = st_gnorm;
    a.critic_step[0] = cstep;
  }
}

__global__ void __launch_bounds__(kWG)
ppo_fused_kernel(smi_ppo_args args) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  FusedCtx c;
  c.a = &args;
  c.F = fused_layout(args.B, args.obs_dim, args.h1, args.h2, args.act_dim,
                     args.critic_h1, args.critic_h2);
  c.sm = sm;
  c.c_loglik = (float)(0.5 * log(2.0 * 3.141592653589793) * (double)args.act_dim);
  c.c_entropy = (float)(0.5 * log(2.0 * 3.141592653589793 * 2.718281828459045) * (double)args.act_dim);
  if (blockIdx.x == 0) policy_wg(c);
  else value_wg(c);
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
  hipLaunchKernelGGL(gae_windows_kernel, dim3(grid), dim3(kWG), lds, stream, a);
  if (n_partials) *n_partials = grid;
  return check_launch("gae_windows_kernel");
}

int launch_ppo_fused(const smi_ppo_args* args, hipStream_t stream) {
  const smi_ppo_args& a = *args;
  if (a.B < 2 || a.B > 256) return set_error(SMI_E_NOFIT, "ppo_fused: B must be in [2, 256]");
  if (a.act_dim < 1 || a.act_dim > 32) return set_error(SMI_E_ARG, "ppo_fused: act_dim in [1,32]");
  const int64_t lds = fused_lds_bytes(a.B, a.obs_dim, a.h1, a.h2, a.act_dim, a.critic_h1,
                                      a.critic_h2);
  if (lds > 160 * 1024) return set_error(SMI_E_NOFIT, "ppo_fused: parameters do not fit LDS");
  hipLaunchKernelGGL(ppo_fused_kernel, dim3(2), dim3(kWG), (size_t)lds, stream, a);
  return check_launch("ppo_fused_kernel");
}

}  // namespace smi
