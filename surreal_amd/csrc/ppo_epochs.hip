// ppo_epochs.hip — the optimisation epochs of PPOLearner._optimize
// (surreal/learner/ppo.py:487-586) on gfx950.
//
//   ppo_fused_kernel        whole epoch loop of one learn() in ONE launch:
//                           workgroup 0 = policy (ref_pol, <= epoch_policy
//                           updates, KL early stop), workgroup 1 = value
//                           (epoch_baseline updates).  Parameters, gradients
//                           and activations stay in LDS for all epochs.
//   ppo_epoch_grad_kernel   data-parallel phase e: this rank's gradient share
//   ppo_epoch_apply_kernel  data-parallel phase e: early stop + Adam after the
//                           cross-rank all-reduce of the exchange buffer
//
// Per-row loss math (ppo_net.py:29-72, ppo.py:194-331) and its analytic
// gradient w.r.t. (mean, std) are written out explicitly; the MLP backward is
// MFMA (smi_device.hpp).
#include "smi_device.hpp"
#include "smi_internal.hpp"

namespace smi {

#ifndef SMI_FWG
#define SMI_FWG 256
#endif
#ifndef SMI_ADAM_PER
#define SMI_ADAM_PER 24
#endif
constexpr int kFWG = SMI_FWG;          // threads of the epoch workgroups (4 waves, 1 per SIMD)
constexpr int kAdamPer = SMI_ADAM_PER; // parameters per thread held in registers

// Developer phase timer (tools/fused_breakdown.py --phases): built only with
// -DSMI_PROF; accumulates wall-clock ticks (100 MHz) per phase and workgroup.
#ifdef SMI_PROF
__device__ unsigned long long g_phase_ticks[2][32];
#define PROF_START() c.prof_t = wall_clock64()
#define PROF(id)                                                          \
  do {                                                                    \
    __syncthreads();                                                      \
    if (threadIdx.x == 0) {                                               \
      const unsigned long long n_ = wall_clock64();                       \
      g_phase_ticks[blockIdx.x & 1][id] += n_ - c.prof_t;                 \
      c.prof_t = n_;                                                      \
    }                                                                     \
  } while (0)
#else
#define PROF_START() (void)0
#define PROF(id) (void)0
#endif

// ---------------------------------------------------------------- layout
struct FusedLayout {
  MlpLayout A, C;
  int Bp, ntiles;
  int ldX, ldH1, ldH, ldO, ldDG, ldOc, ldCH1, ldCH;
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
  F.ldH1 = pad_ld(H1);
  F.ldH = pad_ld(H1 > H2 ? H1 : H2);   // H2 buffer also receives dH1
  F.ldO = pad_small(A);
  F.ldDG = F.ldH;
  int o = 0;
  F.pScr = o; o += 32;                  // 16 doubles of reduction scratch
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
  F.pCol = o; o += round4(6 * A);       // sig, logsig, refsig, reflogsig, gsig, spare
  F.pGS = o; o += round4(kRT * A);      // per-row d loss / d sigma of a tile
  F.pTotal = o;
  F.ldCH1 = pad_ld(cH1);
  F.ldCH = pad_ld(cH1 > cH2 ? cH1 : cH2);
  F.ldOc = pad_small(1);
  o = 0;
  F.vScr = o; o += 32;
  F.vP = o; o += F.C.pcount;
  F.vG = o; o += F.C.pcount;
  F.vX0 = o; o += kRT * F.ldX;
  F.vH1 = o; o += kRT * F.ldCH1;
  F.vH2 = o; o += kRT * F.ldCH;
  F.vOUT = o; o += kRT * F.ldOc;
  F.vDG1 = o; o += kRT * F.ldCH;
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
  return (int64_t)(F.pTotal > F.vTotal ? F.pTotal : F.vTotal) * 4;
}

// exchange-buffer layout (floats) of the data-parallel phases
enum {
  XS_KL = 0, XS_ISW, XS_BL, XS_RBD, XS_RET, XS_SURR, XS_CLIP,
  XS_VSE, XS_VD, XS_VD2, XS_VR, XS_VR2, XS_COUNT = 16
};
struct XLayout { int na, nc, offA, offK, offC, offS, total; };
__host__ __device__ inline XLayout x_layout(int D, int H1, int H2, int A, int cH1, int cH2,
                                            int mode) {
  XLayout X;
  X.na = mlp_layout(D, H1, H2, A, 1).fcount;
  X.nc = mlp_layout(D, cH1, cH2, 1, 0).fcount;
  X.offA = 0;
  X.offK = X.na;
  X.offC = X.offK + (mode == 1 ? X.na : 0);
  X.offS = X.offC + X.nc;
  X.total = X.offS + XS_COUNT;
  return X;
}

// --------------------------------------------------- DiagGauss row helpers
// loglikelihood of ppo_net.py:29-40 with a shared std row (the learner's
// std = exp(log_var) broadcast) and precomputed log(std)
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
// KL(p0 || p1), ppo_net.py:48-62
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

// ------------------------------------------------------------ context
struct FusedCtx {
  const smi_ppo_args* a;
  FusedLayout F;
  float* sm;
  double* scr;
  float c_loglik;   // float(0.5*log(2 pi)*A), as torch rounds the python constant
  float c_entropy;  // float(0.5*log(2 pi e)*A)
  float invB;       // 1 / rows of the (global) batch
  float *P, *G, *refmu, *mu, *act, *beh, *adv, *bpl, *zm, *zs, *rzm, *rzs;
  float *sig, *logsig, *refsig, *reflogsig, *gsig, *gsr;
  unsigned long long prof_t;   // SMI_PROF builds only
};

__device__ inline void ctx_init(FusedCtx& c, const smi_ppo_args& args, float* sm) {
  c.a = &args;
  c.F = fused_layout(args.B, args.obs_dim, args.h1, args.h2, args.act_dim, args.critic_h1,
                     args.critic_h2);
  c.sm = sm;
  c.c_loglik = (float)(0.5 * log(2.0 * 3.141592653589793) * (double)args.act_dim);
  c.c_entropy = (float)(0.5 * log(2.0 * 3.141592653589793 * 2.718281828459045) * (double)args.act_dim);
  const double Bg = args.B_global > 0 ? (double)args.B_global : (double)args.B;
  c.invB = (float)(1.0 / Bg);
  const FusedLayout& F = c.F;
  const int A = args.act_dim;
  c.scr = reinterpret_cast<double*>(sm + F.pScr);
  c.P = sm + F.pP; c.G = sm + F.pG;
  c.refmu = sm + F.pRefMu; c.mu = sm + F.pMu; c.act = sm + F.pAct; c.beh = sm + F.pBeh;
  c.adv = sm + F.pAdv; c.bpl = sm + F.pBp;
  c.zm = sm + F.pZm; c.zs = sm + F.pZs; c.rzm = sm + F.pRZm; c.rzs = sm + F.pRZs;
  c.sig = sm + F.pCol; c.logsig = c.sig + A; c.refsig = c.logsig + A;
  c.reflogsig = c.refsig + A; c.gsig = c.reflogsig + A;
  c.gsr = sm + F.pGS;
}

// actor forward of one 64-row tile into the policy buffers
// Every epoch-loop helper is force-inlined: an out-of-line call passes the
// context structs through scratch and saves/restores registers around it.
#ifndef SMI_INL
#define SMI_INL __device__ __attribute__((always_inline))
#endif

SMI_INL void policy_fwd_tile(const FusedCtx& c, const MlpView& V, int tile,
                                const float* zm, const float* zs) {
  const smi_ppo_args& a = *c.a;
  const FusedLayout& F = c.F;
  float* sm = c.sm;
  const int r0 = tile * kRT;
  const int nr = min(kRT, a.B - r0);
  load_obs_tile<kFWG>(a.obs + (int64_t)r0 * a.obs_stride, a.obs_stride, nr, a.obs_dim,
                a.use_zf ? zm : nullptr, zs, sm + F.pX0, F.ldX);
  __syncthreads();
  dense_fwd<ACT_RELU, kFWG>(sm + F.pX0, F.ldX, V.W1, V.ld1, V.b1, a.obs_dim, a.h1, sm + F.pH1, F.ldH1);
  __syncthreads();
  dense_fwd<ACT_RELU, kFWG>(sm + F.pH1, F.ldH1, V.W2, V.ld2, V.b2, a.h1, a.h2, sm + F.pH2, F.ldH);
  __syncthreads();
  dense_fwd<ACT_TANH, kFWG>(sm + F.pH2, F.ldH, V.W3, V.ld3, V.b3, a.h2, a.act_dim, sm + F.pOUT, F.ldO);
  __syncthreads();
}

// Everything the policy loop needs before its first update: ZFilter column
// stats, per-row actions / behaviour policy / normalised advantages /
// behaviour likelihoods, the reference policy ref_pol (ppo.py:539), and the
// model actor in LDS with zeroed gradients.
SMI_INL void policy_prologue(FusedCtx& c) {
  const smi_ppo_args& a = *c.a;
  const FusedLayout& F = c.F;
  float* sm = c.sm;
  const int A = a.act_dim, B = a.B;
  for (int e = F.pX0 + threadIdx.x; e < F.pRefMu; e += kFWG) sm[e] = 0.f;
  if (a.use_zf) {
    zfilter_colstats<kFWG>(a.zf_sum, a.zf_sumsq, a.zf_count, a.zf_eps, a.obs_dim, c.zm, c.zs);
    zfilter_colstats<kFWG>(a.rzf_sum, a.rzf_sumsq, a.rzf_count, a.zf_eps, a.obs_dim, c.rzm, c.rzs);
  }
  for (int e = threadIdx.x; e < F.Bp * A; e += kFWG) {
    const int r = e / A, j = e - r * A;
    const bool v = r < B;
    c.act[e] = v ? a.actions[(int64_t)r * a.act_stride + j] : 0.f;
    c.beh[r * 2 * A + j] = v ? a.behave[(int64_t)r * a.beh_stride + j] : 0.f;
    c.beh[r * 2 * A + A + j] = v ? a.behave[(int64_t)r * a.beh_stride + A + j] : 1.f;
  }
  // advantage normalisation (ppo.py:413-416): unbiased std, max(std, 1e-4)
  {
    double s1, s2, n;
    if (a.adv_moments) {
      s1 = a.adv_moments[0]; s2 = a.adv_moments[1]; n = a.adv_moments[2];
    } else {
      double l1 = 0.0;
      for (int r = threadIdx.x; r < B; r += kFWG) l1 += (double)a.adv_raw[r];
      s1 = block_sum_d<kFWG>(l1, c.scr);
      n = (double)B;
      const double mean = s1 / n;
      double l2 = 0.0;
      for (int r = threadIdx.x; r < B; r += kFWG) {
        const double d = (double)a.adv_raw[r] - mean;
        l2 += d * d;
      }
      s2 = block_sum_d<kFWG>(l2, c.scr) + n * mean * mean;
    }
    const double mean_d = s1 / n;
    const double var_d = (s2 - n * mean_d * mean_d) / (n - 1.0);
    const float mean_f = (float)mean_d;
    const float std_f = (float)sqrt(var_d > 0.0 ? var_d : 0.0);
    const float denom = std_f > 1e-4f ? std_f : 1e-4f;
    for (int r = threadIdx.x; r < F.Bp; r += kFWG) {
      float v = 0.f;
      if (r < B) v = a.norm_adv ? (a.adv_raw[r] - mean_f) / denom : a.adv_raw[r];
      c.adv[r] = v;
      if (a.adv_out && r < B) a.adv_out[r] = v;
    }
  }
  __syncthreads();
  for (int r = threadIdx.x; r < F.Bp; r += kFWG) {
    float v = 1.f;
    if (r < B) {
      const float* p = c.beh + r * 2 * A;
      v = fmaxf(expf(dg_loglik_rowstd(c.act + r * A, p, p + A, A, c.c_loglik)), 1e-5f);
    }
    c.bpl[r] = v;
  }
  // reference policy with ref_target_model (its own ZFilter)
  mlp_load_lds<kFWG>(F.A, a.ref_actor, c.P);
  {
    const MlpView V = view_padded(F.A, c.P);
    for (int j = threadIdx.x; j < A; j += kFWG) {
      c.refsig[j] = expf(V.lv[j]);
      c.reflogsig[j] = logf(c.refsig[j]);
    }
    for (int tile = 0; tile < F.ntiles; ++tile) {
      policy_fwd_tile(c, V, tile, c.rzm, c.rzs);
      for (int e = threadIdx.x; e < kRT * A; e += kFWG) {
        const int r = e / A, j = e - r * A;
        c.refmu[(tile * kRT + r) * A + j] = sm[F.pOUT + r * F.ldO + j];
      }
      __syncthreads();
    }
  }
  mlp_load_lds<kFWG>(F.A, a.actor, c.P);
  for (int i = threadIdx.x; i < F.A.pcount; i += kFWG) c.G[i] = 0.f;
  __syncthreads();
}

// Forward of every tile with the current parameters.  Leaves mu (curr_pol
// means) in LDS and returns the block sums of KL(ref || curr) (ppo.py:553-554)
// and of the final-statistics terms (ppo.py:568-575).
struct PolicySums { float kl, isw, bl, rbd, ret; };
SMI_INL PolicySums policy_forward_all(FusedCtx& c, const MlpView& V) {
  const smi_ppo_args& a = *c.a;
  const FusedLayout& F = c.F;
  const int A = a.act_dim, B = a.B;
  for (int j = threadIdx.x; j < A; j += kFWG) {
    c.sig[j] = expf(V.lv[j]);                  // builders.py:127
    c.logsig[j] = logf(c.sig[j]);
  }
  __syncthreads();
  float klp = 0.f, iswp = 0.f, blp = 0.f, rbdp = 0.f, retp = 0.f;
  for (int tile = 0; tile < F.ntiles; ++tile) {
    policy_fwd_tile(c, V, tile, c.zm, c.zs);
    PROF(8);
    for (int e = threadIdx.x; e < kRT * A; e += kFWG) {
      const int r = e / A, j = e - r * A;
      c.mu[(tile * kRT + r) * A + j] = c.sm[F.pOUT + r * F.ldO + j];
    }
    __syncthreads();
    for (int r = threadIdx.x; r < kRT; r += kFWG) {
      const int gr = tile * kRT + r;
      if (gr < B) {
        const float* m = c.mu + gr * A;
        klp += dg_kl(c.refmu + gr * A, c.refsig, m, c.sig, A);
        const float bl = c.bpl[gr];
        const float cl = fmaxf(expf(dg_loglik(c.act + gr * A, m, c.sig, c.logsig, A, c.c_loglik)), 1e-5f);
        iswp += cl / (bl + 1e-4f);
        blp += bl;
        const float* p = c.beh + gr * 2 * A;
        rbdp += dg_kl(c.refmu + gr * A, c.refsig, p, p + A, A);
        retp += a.ret[gr];
      }
    }
  }
  PROF(9);
  PolicySums s;
  s.kl = block_sum_f<kFWG>(klp, c.scr);
  s.isw = block_sum_f<kFWG>(iswp, c.scr);
  s.bl = block_sum_f<kFWG>(blp, c.scr);
  s.rbd = block_sum_f<kFWG>(rbdp, c.scr);
  s.ret = block_sum_f<kFWG>(retp, c.scr);
  return s;
}

// Per-row loss gradient w.r.t. (mean, std) and the MLP backward of one tile,
// accumulated into G (LDS) and gsig.
//   surr_w = 1: clip (mode 0, ppo.py:209-217) or adapt (mode 1, ppo.py:267-271)
//              surrogate term, weight invB per row
//   gkl    = d loss / d KL_i of the adapt penalty term (0 = none)
// When recompute is false the tile's activations must still be in LDS.
SMI_INL void policy_loss_bwd_tile(FusedCtx& c, const MlpView& V, int tile, bool recompute,
                                     float surr_w, float gkl, float clip_lo, float clip_hi,
                                     float* p_surr, float* p_clip) {
  const smi_ppo_args& a = *c.a;
  const FusedLayout& F = c.F;
  float* sm = c.sm;
  const int A = a.act_dim, B = a.B;
  if (recompute) policy_fwd_tile(c, V, tile, c.zm, c.zs);
  float* dOut = sm + F.pDG2;
  for (int r = threadIdx.x; r < kRT; r += kFWG) {
    const int gr = tile * kRT + r;
    float* dz = dOut + r * F.ldO;
    if (gr >= B) {
      for (int j = 0; j < F.ldO; ++j) dz[j] = 0.f;
      for (int j = 0; j < A; ++j) c.gsr[r * A + j] = 0.f;
      continue;
    }
    const float* m = sm + F.pOUT + r * F.ldO;        // this tile's forward output
    const float* ac = c.act + gr * A;
    const float ll = dg_loglik(ac, m, c.sig, c.logsig, A, c.c_loglik);
    const float ex = expf(ll);
    const float lp = fmaxf(ex, 1e-5f);               // likelihood clamp (ppo_net.py:46)
    const float bp = c.bpl[gr];
    const float av = c.adv[gr];
    float g_lp = 0.f;
    if (surr_w != 0.f) {
      if (a.mode == 0) {
        const float ratio = lp / bp;
        const float cr = fminf(fmaxf(ratio, clip_lo), clip_hi);
        const float surr = -ratio * av;
        const float csur = -cr * av;
        *p_surr += surr;
        *p_clip += fmaxf(surr, csur);
        // max() routes the gradient to the surrogate unless the clipped one is
        // strictly larger, in which case the ratio is outside the clamp range
        // and the gradient is 0 either way.
        g_lp = ((surr >= csur) ? -(c.invB * av) : 0.f) / bp;
      } else {
        const float bpc = fmaxf(bp, 1e-2f);
        *p_surr += av * (lp / bpc);
        g_lp = (-c.invB * av) / bpc;
      }
    }
    const float g_ll = (ex >= 1e-5f) ? g_lp * ex : 0.f;   // clamp + exp backward
    for (int j = 0; j < A; ++j) {
      const float s1 = c.sig[j];
      const float u = (ac[j] - m[j]) / s1;
      float gmu = g_ll * (u / s1);                       // d loglik / d mean
      float gsd = g_ll * (u * u / s1 - 1.f / s1);        // d loglik / d std
      if (gkl != 0.f) {
        const float d = c.refmu[gr * A + j] - m[j];
        gmu += gkl * (-d / (s1 * s1));                   // d KL(ref||cur) / d mean
        gsd += gkl * (1.f / s1 - (c.refsig[j] * c.refsig[j] + d * d) / (s1 * s1 * s1));
      }
      c.gsr[r * A + j] = gsd;
      dz[j] = gmu * (1.f - m[j] * m[j]);               // tanh backward
    }
    for (int j = A; j < F.ldO; ++j) dz[j] = 0.f;
  }
  __syncthreads();
  PROF(10);
  for (int j = threadIdx.x; j < A; j += kFWG) {
    float s = 0.f;
    for (int r = 0; r < kRT; ++r) s += c.gsr[r * A + j];
    c.gsig[j] += s;
  }
  // backward through Linear-ReLU-Linear-ReLU-Linear (dW3, dH2 | dW2, dH1 | dW1)
  float* X0 = sm + F.pX0; float* H1 = sm + F.pH1; float* H2 = sm + F.pH2;
  float* DG1 = sm + F.pDG1;
  const MlpLayout& L = F.A;
  float* G = c.G;
  PROF(11);
  dense_bwd_dw<kFWG>(dOut, F.ldO, H2, F.ldH, a.h2, A, G + L.pW3, L.ld3, G + L.pb3);
  dense_bwd_dx<ACT_RELU, kFWG>(dOut, F.ldO, V.W3, V.ld3, a.h2, A, H2, F.ldH, DG1, F.ldDG);
  __syncthreads();
  dense_bwd_dw<kFWG>(DG1, F.ldDG, H1, F.ldH1, a.h1, a.h2, G + L.pW2, L.ld2, G + L.pb2);
  dense_bwd_dx<ACT_RELU, kFWG>(DG1, F.ldDG, V.W2, V.ld2, a.h1, a.h2, H1, F.ldH1, H2, F.ldH);
  __syncthreads();
  dense_bwd_dw<kFWG>(H2, F.ldH, X0, F.ldX, a.obs_dim, a.h1, G + L.pW1, L.ld1, G + L.pb1);
  __syncthreads();
  PROF(12);
}

// log_var gradient: std = exp(log_var) * ones -> sum over rows of g_std * std
__device__ inline void policy_finish_logvar_grad(FusedCtx& c) {
  for (int j = threadIdx.x; j < c.a->act_dim; j += kFWG) c.G[c.F.A.plv + j] = c.gsig[j] * c.sig[j];
  __syncthreads();
}

// Adam on a padded LDS parameter image (torch.optim.Adam single-tensor path):
//   m.lerp_(g, 1-b1); v.mul_(b2).addcmul_(g, g, 1-b2);
//   p.addcdiv_(m, v.sqrt()/sqrt(1-b2^t) + eps, value=-lr/(1-b1^t))
// The Adam moments of the parameters a thread owns (flat index
// threadIdx.x + u*kFWG) stay in registers for the whole epoch loop, with the
// LDS index of each parameter precomputed: no global traffic and no index
// arithmetic per update.  Loaded once per launch, stored once at the end.
struct AdamRegs {
  float m[kAdamPer], v[kAdamPer];
  int pi[kAdamPer];

  SMI_INL void load(const MlpLayout& L, const float* __restrict__ gm,
                       const float* __restrict__ gv) {
#pragma unroll
    for (int u = 0; u < kAdamPer; ++u) {
      const int i = threadIdx.x + u * kFWG;
      const bool ok = i < L.fcount;
      m[u] = ok ? gm[i] : 0.f;
      v[u] = ok ? gv[i] : 0.f;
      pi[u] = ok ? mlp_flat_to_pad(L, i) : 0;
    }
  }
  SMI_INL void store(const MlpLayout& L, float* __restrict__ gm, float* __restrict__ gv) const {
#pragma unroll
    for (int u = 0; u < kAdamPer; ++u) {
      const int i = threadIdx.x + u * kFWG;
      if (i < L.fcount) { gm[i] = m[u]; gv[i] = v[u]; }
    }
  }
  // global L2 norm of the gradient image (fp64 accumulation)
  SMI_INL float grad_norm(const MlpLayout& L, const float* G, double* scr) const {
    double s = 0.0;
#pragma unroll
    for (int u = 0; u < kAdamPer; ++u) {
      const int i = threadIdx.x + u * kFWG;
      if (i < L.fcount) {
        const float g = G[pi[u]];
        s += (double)g * (double)g;
      }
    }
    return (float)sqrt(block_sum_d<kFWG>(s, scr));
  }
  // torch.optim.Adam single-tensor path on the padded LDS image P:
  //   m.lerp_(g, 1-b1); v.mul_(b2).addcmul_(g, g, 1-b2);
  //   p.addcdiv_(m, v.sqrt()/sqrt(1-b2^t) + eps, value=-lr/(1-b1^t))
  SMI_INL void step(const MlpLayout& L, float* P, const float* G, int t, float lr,
                       float beta1, float beta2, float eps, float wd, float coef) {
    __syncthreads();
    const double bc1 = 1.0 - pow((double)beta1, (double)t);
    const double bc2 = 1.0 - pow((double)beta2, (double)t);
    const float step_size = (float)((double)lr / bc1);
    const float bc2_sqrt = (float)sqrt(bc2);
    const float w1 = (float)(1.0 - (double)beta1);
    const float w2 = (float)(1.0 - (double)beta2);
#pragma unroll
    for (int u = 0; u < kAdamPer; ++u) {
      const int i = threadIdx.x + u * kFWG;
      if (i < L.fcount) {
        float g = G[pi[u]] * coef;
        float p = P[pi[u]];
        if (wd != 0.f) g = g + wd * p;
        float mi = m[u], vi = v[u];
        mi = mi + w1 * (g - mi);
        vi = vi * beta2 + (w2 * g) * g;
        const float denom = sqrtf(vi) / bc2_sqrt + eps;
        P[pi[u]] = p + (-step_size) * (mi / denom);
        m[u] = mi; v[u] = vi;
      }
    }
    __syncthreads();
  }
};

__device__ inline float clip_coef(float norm, float max_norm) {
  const float cc = max_norm / (norm + 1e-6f);       // clip_grad_norm_
  return cc < 1.f ? cc : 1.f;
}

__device__ inline float entropy_of(const FusedCtx& c) {
  float ent = 0.f;
  for (int j = 0; j < c.a->act_dim; ++j) ent += c.logsig[j];
  return 0.5f * ent + c.c_entropy;                  // ppo_net.py:64-72 (constant per row)
}

__device__ inline bool adapt_penalty_on(float kl, double kl_target) {
  return (double)kl - 2.0 * kl_target > 0.0;        // ppo.py:275 (python float compare)
}

// ============================================================ fused kernel
SMI_INL void policy_wg(FusedCtx& c) {
  const smi_ppo_args& a = *c.a;
  const FusedLayout& F = c.F;
  const int A = a.act_dim;
  const float clip_lo = a.hyper[SMI_HYPX_CLIP_LO];
  const float clip_hi = a.hyper[SMI_HYPX_CLIP_HI];
  const float beta = a.hyper[SMI_HYP_BETA];
  const float lr = a.hyper[SMI_HYP_LR_ACTOR];
  PROF_START();
  policy_prologue(c);
  PROF(0);
  const MlpView V = view_padded(F.A, c.P);
  float st_surr = 0.f, st_clip = 0.f, st_kladapt = 0.f, st_ent = 0.f, st_gnorm = 0.f;
  float st_klad = 0.f, pol_kl = 0.f;
  int epochs_run = 0;
  int astep = a.actor_step[0];
  AdamRegs opt;
  opt.load(F.A, a.actor_m, a.actor_v);
  PolicySums fin;
  const int E = a.epoch_policy;
  for (int e = 0; e <= E; ++e) {
    fin = policy_forward_all(c, V);
    PROF(1);
    const float kl = fin.kl * c.invB;
    if (e > 0) {
      pol_kl = kl;                                            // ppo.py:553-555
      if ((double)kl > a.kl_target * 4.0) break;              // ppo.py:556-557
    }
    if (e == E) break;
    float gkl = 0.f;
    if (a.mode == 1) {
      float coef = beta;
      if (adapt_penalty_on(kl, a.kl_target))
        coef = beta + a.kl_cutoff_coeff * 2.f * (kl - (float)(2.0 * a.kl_target));
      gkl = coef * c.invB;
    }
    for (int j = threadIdx.x; j < A; j += kFWG) c.gsig[j] = 0.f;
    float p_surr = 0.f, p_clip = 0.f;
    for (int tile = 0; tile < F.ntiles; ++tile)
      policy_loss_bwd_tile(c, V, tile, F.ntiles > 1, 1.f, gkl, clip_lo, clip_hi, &p_surr, &p_clip);
    policy_finish_logvar_grad(c);
    PROF(2);
    const float tot_surr = block_sum_f<kFWG>(p_surr, c.scr);
    const float tot_clip = block_sum_f<kFWG>(p_clip, c.scr);
    if (a.mode == 0) {
      st_surr = tot_surr * c.invB;
      st_clip = tot_clip * c.invB;
    } else {
      const float surr = -(tot_surr * c.invB);
      float loss = surr + beta * kl;
      if (adapt_penalty_on(kl, a.kl_target)) {
        const float d = kl - (float)(2.0 * a.kl_target);
        loss = loss + a.kl_cutoff_coeff * (d * d);
      }
      st_surr = surr;
      st_kladapt = loss;
      st_klad = kl;
    }
    st_ent = entropy_of(c);
    PROF(3);
    const float norm = opt.grad_norm(F.A, c.G, c.scr);          // clip_grad_norm_ (ppo.py:243)
    float coef = 1.f;
    if (a.clip_actor_grad) {
      coef = clip_coef(norm, a.actor_max_norm);
      st_gnorm = norm;
    }
    PROF(4);
    ++astep;
    opt.step(F.A, c.P, c.G, astep, lr, a.beta1, a.beta2, a.adam_eps, a.actor_wd, coef);  // :247
    for (int i = threadIdx.x; i < F.A.pcount; i += kFWG) c.G[i] = 0.f;
    ++epochs_run;
    __syncthreads();
    PROF(5);
  }
  mlp_store_flat<kFWG>(F.A, c.P, a.actor);
  opt.store(F.A, a.actor_m, a.actor_v);
  PROF(6);
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
    st[SMI_ST_AVG_RETURN] = fin.ret * c.invB;
    st[SMI_ST_AVG_LOG_SIG] = lvs / (float)A;
    st[SMI_ST_AVG_BEHAVE_LIK] = fin.bl * c.invB;
    st[SMI_ST_AVG_IS_WEIGHT] = fin.isw * c.invB;
    st[SMI_ST_REF_BEHAVE_DIFF] = fin.rbd * c.invB;
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

// value workgroup: one critic epoch's forward + loss + backward into G over all
// tiles (ppo.py:311-331), returning the double sums used by the statistics
struct ValueSums { double se, d, d2, r, r2; };
SMI_INL ValueSums value_grad_epoch(const smi_ppo_args& a, const FusedLayout& F, float* sm,
                                      const MlpView& V, float invB) {
  const MlpLayout& L = F.C;
  double* scr = reinterpret_cast<double*>(sm + F.vScr);
  float* G = sm + F.vG;
  float* X0 = sm + F.vX0; float* H1 = sm + F.vH1; float* H2 = sm + F.vH2;
  float* OUT = sm + F.vOUT; float* DG1 = sm + F.vDG1; float* DG2 = sm + F.vDG2;
  float* ret = sm + F.vRet; float* Vv = sm + F.vV;
  float* zm = sm + F.vZm; float* zs = sm + F.vZs;
  const int ldH1 = F.ldCH1, ldH = F.ldCH, ldO = F.ldOc;
  const int B = a.B;
  for (int tile = 0; tile < F.ntiles; ++tile) {
    const int r0 = tile * kRT, nr = min(kRT, B - r0);
    load_obs_tile<kFWG>(a.obs + (int64_t)r0 * a.obs_stride, a.obs_stride, nr, a.obs_dim,
                  a.use_zf ? zm : nullptr, zs, X0, F.ldX);
    __syncthreads();
    dense_fwd<ACT_RELU, kFWG>(X0, F.ldX, V.W1, V.ld1, V.b1, a.obs_dim, a.critic_h1, H1, ldH1);
    __syncthreads();
    dense_fwd<ACT_RELU, kFWG>(H1, ldH1, V.W2, V.ld2, V.b2, a.critic_h1, a.critic_h2, H2, ldH);
    __syncthreads();
    dense_fwd<ACT_NONE, kFWG>(H2, ldH, V.W3, V.ld3, V.b3, a.critic_h2, 1, OUT, ldO);
    __syncthreads();
    // d/dV mean((V - R)^2) = 2 (V - R) / B   (ppo.py:326)
    for (int r = threadIdx.x; r < kRT; r += kFWG) {
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
    dense_bwd_dw<kFWG>(DG2, ldO, H2, ldH, a.critic_h2, 1, G + L.pW3, L.ld3, G + L.pb3);
    dense_bwd_dx<ACT_RELU, kFWG>(DG2, ldO, V.W3, V.ld3, a.critic_h2, 1, H2, ldH, DG1, ldH);
    __syncthreads();
    dense_bwd_dw<kFWG>(DG1, ldH, H1, ldH1, a.critic_h1, a.critic_h2, G + L.pW2, L.ld2, G + L.pb2);
    dense_bwd_dx<ACT_RELU, kFWG>(DG1, ldH, V.W2, V.ld2, a.critic_h1, a.critic_h2, H1, ldH1, H2, ldH);
    __syncthreads();
    dense_bwd_dw<kFWG>(H2, ldH, X0, F.ldX, a.obs_dim, a.critic_h1, G + L.pW1, L.ld1, G + L.pb1);
    __syncthreads();
  }
  double l_se = 0.0, l_d = 0.0, l_d2 = 0.0, l_r = 0.0, l_r2 = 0.0;
  for (int r = threadIdx.x; r < B; r += kFWG) {
    const float e = Vv[r] - ret[r];
    const double d = (double)ret[r] - (double)Vv[r];
    l_se += (double)(e * e);
    l_d += d; l_d2 += d * d;
    l_r += (double)ret[r]; l_r2 += (double)ret[r] * (double)ret[r];
  }
  ValueSums s;
  s.se = block_sum_d<kFWG>(l_se, scr);
  s.d = block_sum_d<kFWG>(l_d, scr);
  s.d2 = block_sum_d<kFWG>(l_d2, scr);
  s.r = block_sum_d<kFWG>(l_r, scr);
  s.r2 = block_sum_d<kFWG>(l_r2, scr);
  return s;
}

__device__ inline float unbiased_var(double s, double s2, double n) {
  const double mean = s / n;
  return (float)((s2 - n * mean * mean) / (n - 1.0));
}

SMI_INL void value_prologue(const smi_ppo_args& a, const FusedLayout& F, float* sm) {
  for (int e = F.vX0 + threadIdx.x; e < F.vRet; e += kFWG) sm[e] = 0.f;
  if (a.use_zf)
    zfilter_colstats<kFWG>(a.zf_sum, a.zf_sumsq, a.zf_count, a.zf_eps, a.obs_dim, sm + F.vZm, sm + F.vZs);
  for (int r = threadIdx.x; r < F.Bp; r += kFWG) sm[F.vRet + r] = r < a.B ? a.ret[r] : 0.f;
  mlp_load_lds<kFWG>(F.C, a.critic, sm + F.vP);
  for (int i = threadIdx.x; i < F.C.pcount; i += kFWG) sm[F.vG + i] = 0.f;
  __syncthreads();
}

SMI_INL void value_wg(FusedCtx& c) {
  const smi_ppo_args& a = *c.a;
  const FusedLayout& F = c.F;
  float* sm = c.sm;
  double* scr = reinterpret_cast<double*>(sm + F.vScr);
  const MlpLayout& L = F.C;
  float* P = sm + F.vP;
  float* G = sm + F.vG;
  const float lr = a.hyper[SMI_HYP_LR_CRITIC];
  PROF_START();
  value_prologue(a, F, sm);
  PROF(0);
  const MlpView V = view_padded(L, P);
  float st_loss = 0.f, st_ev = 0.f, st_gnorm = 0.f;
  int cstep = a.critic_step[0];
  AdamRegs opt;
  opt.load(L, a.critic_m, a.critic_v);
  const double n = (double)a.B;
  for (int e = 0; e < a.epoch_baseline; ++e) {
    const ValueSums s = value_grad_epoch(a, F, sm, V, c.invB);
    PROF(2);
    st_loss = (float)(s.se / n);
    st_ev = 1.f - unbiased_var(s.d, s.d2, n) / unbiased_var(s.r, s.r2, n);   // ppo.py:325
    const float norm = opt.grad_norm(L, G, scr);
    PROF(4);
    float coef = 1.f;
    if (a.clip_critic_grad) {
      coef = clip_coef(norm, a.critic_max_norm);
      st_gnorm = norm;
    }
    ++cstep;
    opt.step(L, P, G, cstep, lr, a.beta1, a.beta2, a.adam_eps, a.critic_wd, coef);
    for (int i = threadIdx.x; i < L.pcount; i += kFWG) G[i] = 0.f;
    __syncthreads();
    PROF(5);
  }
  mlp_store_flat<kFWG>(L, P, a.critic);
  opt.store(L, a.critic_m, a.critic_v);
  PROF(6);
  if (threadIdx.x == 0) {
    a.stats[SMI_ST_VAL_LOSS] = st_loss;
    a.stats[SMI_ST_VAL_EXPL_VAR] = st_ev;
    a.stats[SMI_ST_GRAD_NORM_CRITIC] = st_gnorm;
    a.critic_step[0] = cstep;
  }
}

__global__ void __launch_bounds__(kFWG)
ppo_fused_kernel(smi_ppo_args args) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  FusedCtx c;
  ctx_init(c, args, sm);
  if (blockIdx.x == 0) policy_wg(c);
  else value_wg(c);
}

// ================================================== data-parallel phases
// dp_state: [0] policy stopped, [1] policy updates applied
__global__ void __launch_bounds__(kFWG)
ppo_epoch_grad_kernel(smi_ppo_args args, int e) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  FusedCtx c;
  ctx_init(c, args, sm);
  const smi_ppo_args& a = args;
  const FusedLayout& F = c.F;
  const XLayout X = x_layout(a.obs_dim, a.h1, a.h2, a.act_dim, a.critic_h1, a.critic_h2, a.mode);
  float* xs = a.xbuf + X.offS;
  if (blockIdx.x == 0) {
    if (a.dp_state[0] != 0 || e > a.epoch_policy) {
      // stopped: contribute zeros so the all-reduced sums stay defined
      for (int i = threadIdx.x; i < X.offC; i += kFWG) a.xbuf[i] = 0.f;
      if (threadIdx.x == 0)
        for (int k = XS_KL; k <= XS_CLIP; ++k) xs[k] = 0.f;
      return;
    }
    const float clip_lo = a.hyper[SMI_HYPX_CLIP_LO];
    const float clip_hi = a.hyper[SMI_HYPX_CLIP_HI];
    policy_prologue(c);
    const MlpView V = view_padded(F.A, c.P);
    const PolicySums s = policy_forward_all(c, V);
    float p_surr = 0.f, p_clip = 0.f;
    if (e < a.epoch_policy) {
      // surrogate gradient (the adapt KL term goes to its own slot: its weight
      // depends on the GLOBAL KL, known only after the all-reduce)
      for (int j = threadIdx.x; j < a.act_dim; j += kFWG) c.gsig[j] = 0.f;
      for (int tile = 0; tile < F.ntiles; ++tile)
        policy_loss_bwd_tile(c, V, tile, F.ntiles > 1, 1.f, 0.f, clip_lo, clip_hi, &p_surr, &p_clip);
      policy_finish_logvar_grad(c);
      for (int i = threadIdx.x; i < F.A.fcount; i += kFWG)
        a.xbuf[X.offA + i] = c.G[mlp_flat_to_pad(F.A, i)];
      if (a.mode == 1) {
        __syncthreads();
        for (int i = threadIdx.x; i < F.A.pcount; i += kFWG) c.G[i] = 0.f;
        for (int j = threadIdx.x; j < a.act_dim; j += kFWG) c.gsig[j] = 0.f;
        float d0 = 0.f, d1 = 0.f;
        for (int tile = 0; tile < F.ntiles; ++tile)
          policy_loss_bwd_tile(c, V, tile, true, 0.f, c.invB, clip_lo, clip_hi, &d0, &d1);
        policy_finish_logvar_grad(c);
        for (int i = threadIdx.x; i < F.A.fcount; i += kFWG)
          a.xbuf[X.offK + i] = c.G[mlp_flat_to_pad(F.A, i)];
      }
    } else {
      for (int i = threadIdx.x; i < X.offC; i += kFWG) a.xbuf[i] = 0.f;
    }
    const float t_surr = block_sum_f<kFWG>(p_surr, c.scr);
    const float t_clip = block_sum_f<kFWG>(p_clip, c.scr);
    if (threadIdx.x == 0) {
      xs[XS_KL] = s.kl; xs[XS_ISW] = s.isw; xs[XS_BL] = s.bl; xs[XS_RBD] = s.rbd;
      xs[XS_RET] = s.ret; xs[XS_SURR] = t_surr; xs[XS_CLIP] = t_clip;
    }
  } else {
    if (e >= a.epoch_baseline) {
      for (int i = threadIdx.x; i < X.nc; i += kFWG) a.xbuf[X.offC + i] = 0.f;
      if (threadIdx.x == 0)
        for (int k = XS_VSE; k <= XS_VR2; ++k) xs[k] = 0.f;
      return;
    }
    value_prologue(a, F, sm);
    const MlpView V = view_padded(F.C, sm + F.vP);
    const ValueSums s = value_grad_epoch(a, F, sm, V, c.invB);
    for (int i = threadIdx.x; i < F.C.fcount; i += kFWG)
      a.xbuf[X.offC + i] = sm[F.vG + mlp_flat_to_pad(F.C, i)];
    if (threadIdx.x == 0) {
      xs[XS_VSE] = (float)s.se; xs[XS_VD] = (float)s.d; xs[XS_VD2] = (float)s.d2;
      xs[XS_VR] = (float)s.r; xs[XS_VR2] = (float)s.r2;
    }
  }
}

// Adam over a flat global parameter vector; g_i = (ga[i] + kc * gk[i]) * coef
__device__ void adam_global(float* p, const float* ga, const float* gk, float kc, float coef,
                            float* m, float* v, int n, int t, float lr, float beta1, float beta2,
                            float eps, float wd) {
  const double bc1 = 1.0 - pow((double)beta1, (double)t);
  const double bc2 = 1.0 - pow((double)beta2, (double)t);
  const float step_size = (float)((double)lr / bc1);
  const float bc2_sqrt = (float)sqrt(bc2);
  const float w1 = (float)(1.0 - (double)beta1);
  const float w2 = (float)(1.0 - (double)beta2);
  for (int i = threadIdx.x; i < n; i += kWG) {
    float g = gk ? ga[i] + kc * gk[i] : ga[i];
    g = g * coef;
    float pi = p[i];
    if (wd != 0.f) g = g + wd * pi;
    float mi = m[i], vi = v[i];
    mi = mi + w1 * (g - mi);
    vi = vi * beta2 + (w2 * g) * g;
    const float denom = sqrtf(vi) / bc2_sqrt + eps;
    p[i] = pi + (-step_size) * (mi / denom);
    m[i] = mi; v[i] = vi;
  }
}

__device__ float sumsq_global(const float* ga, const float* gk, float kc, int n, double* scr) {
  double s = 0.0;
  for (int i = threadIdx.x; i < n; i += kWG) {
    const float g = gk ? ga[i] + kc * gk[i] : ga[i];
    s += (double)g * (double)g;
  }
  return (float)sqrt(block_sum_d<kWG>(s, scr));
}

__global__ void __launch_bounds__(kWG)
ppo_epoch_apply_kernel(smi_ppo_args a, int e) {
  __shared__ double scr[kNW];
  __shared__ int s_stop;
  const XLayout X = x_layout(a.obs_dim, a.h1, a.h2, a.act_dim, a.critic_h1, a.critic_h2, a.mode);
  const float* xs = a.xbuf + X.offS;
  const double Bg = a.B_global > 0 ? (double)a.B_global : (double)a.B;
  const float invB = (float)(1.0 / Bg);
  const int E = a.epoch_policy;
  float* st = a.stats;
  if (threadIdx.x == 0) s_stop = a.dp_state[0];
  __syncthreads();
  // ---------------- policy
  if (!s_stop && e <= E) {
    const float kl = xs[XS_KL] * invB;
    bool last = false;
    if (e > 0) {
      if ((double)kl > a.kl_target * 4.0) last = true;         // ppo.py:556
    }
    if (e == E) last = true;
    if (last) {
      if (threadIdx.x == 0) {
        if (e > 0) st[SMI_ST_POL_KL] = kl;
        st[SMI_ST_AVG_RETURN] = xs[XS_RET] * invB;
        st[SMI_ST_AVG_BEHAVE_LIK] = xs[XS_BL] * invB;
        st[SMI_ST_AVG_IS_WEIGHT] = xs[XS_ISW] * invB;
        st[SMI_ST_REF_BEHAVE_DIFF] = xs[XS_RBD] * invB;
        const MlpLayout LA = mlp_layout(a.obs_dim, a.h1, a.h2, a.act_dim, 1);
        float lvs = 0.f;
        for (int j = 0; j < a.act_dim; ++j) lvs += a.actor[LA.flv + j];
        st[SMI_ST_AVG_LOG_SIG] = lvs / (float)a.act_dim;
        st[SMI_ST_EPOCHS_RUN] = (float)a.dp_state[1];
        if (a.kl_record && a.kl_count) {
          const int k = a.kl_count[0];
          if (k < a.kl_capacity) a.kl_record[k] = st[SMI_ST_POL_KL];
          a.kl_count[0] = k + 1;
        }
        a.dp_state[0] = 1;
      }
    } else {
      if (e > 0 && threadIdx.x == 0) st[SMI_ST_POL_KL] = kl;
      const float beta = a.hyper[SMI_HYP_BETA];
      float kc = 0.f;
      if (a.mode == 1) {
        kc = beta;
        if (adapt_penalty_on(kl, a.kl_target))
          kc = beta + a.kl_cutoff_coeff * 2.f * (kl - (float)(2.0 * a.kl_target));
      }
      const float* ga = a.xbuf + X.offA;
      const float* gk = a.mode == 1 ? a.xbuf + X.offK : nullptr;
      // entropy of learn_pol (before this update; constant per row, ppo_net.py:64-72)
      if (threadIdx.x == 0) {
        const MlpLayout LA = mlp_layout(a.obs_dim, a.h1, a.h2, a.act_dim, 1);
        const float c_ent = (float)(0.5 * log(2.0 * 3.141592653589793 * 2.718281828459045) *
                                    (double)a.act_dim);
        float ent = 0.f;
        for (int j = 0; j < a.act_dim; ++j) ent += logf(expf(a.actor[LA.flv + j]));
        st[SMI_ST_ENTROPY] = 0.5f * ent + c_ent;
      }
      __syncthreads();
      const float norm = sumsq_global(ga, gk, kc, X.na, scr);
      float coef = 1.f;
      if (a.clip_actor_grad) coef = clip_coef(norm, a.actor_max_norm);
      const int t = a.actor_step[0] + 1;
      adam_global(a.actor, ga, gk, kc, coef, a.actor_m, a.actor_v, X.na, t,
                  a.hyper[SMI_HYP_LR_ACTOR], a.beta1, a.beta2, a.adam_eps, a.actor_wd);
      __syncthreads();
      if (threadIdx.x == 0) {
        a.actor_step[0] = t;
        a.dp_state[1] += 1;
        if (a.mode == 0) {
          st[SMI_ST_SURR_LOSS] = xs[XS_SURR] * invB;
          st[SMI_ST_CLIP_SURR_LOSS] = xs[XS_CLIP] * invB;
        } else {
          const float surr = -(xs[XS_SURR] * invB);
          float loss = surr + beta * kl;
          if (adapt_penalty_on(kl, a.kl_target)) {
            const float d = kl - (float)(2.0 * a.kl_target);
            loss = loss + a.kl_cutoff_coeff * (d * d);
          }
          st[SMI_ST_SURR_LOSS] = surr;
          st[SMI_ST_KL_LOSS_ADAPT] = loss;
          st[SMI_ST_POL_KL_ADAPT] = kl;
        }
        if (a.clip_actor_grad) st[SMI_ST_GRAD_NORM_ACTOR] = norm;
      }
    }
  }
  __syncthreads();
  // ---------------- value
  if (e < a.epoch_baseline) {
    const float* gc = a.xbuf + X.offC;
    const float norm = sumsq_global(gc, nullptr, 0.f, X.nc, scr);
    float coef = 1.f;
    if (a.clip_critic_grad) coef = clip_coef(norm, a.critic_max_norm);
    const int t = a.critic_step[0] + 1;
    adam_global(a.critic, gc, nullptr, 0.f, coef, a.critic_m, a.critic_v, X.nc, t,
                a.hyper[SMI_HYP_LR_CRITIC], a.beta1, a.beta2, a.adam_eps, a.critic_wd);
    __syncthreads();
    if (threadIdx.x == 0) {
      a.critic_step[0] = t;
      st[SMI_ST_VAL_LOSS] = (float)((double)xs[XS_VSE] / Bg);
      st[SMI_ST_VAL_EXPL_VAR] = 1.f - unbiased_var(xs[XS_VD], xs[XS_VD2], Bg) /
                                      unbiased_var(xs[XS_VR], xs[XS_VR2], Bg);
      if (a.clip_critic_grad) st[SMI_ST_GRAD_NORM_CRITIC] = norm;
    }
  }
}

// ============================================================ launchers
static int fused_check(const smi_ppo_args& a, int64_t* lds_out) {
  if (a.B < 1 || a.B > 256) return set_error(SMI_E_NOFIT, "ppo epochs: B must be in [1, 256]");
  if (a.act_dim < 1 || a.act_dim > 32) return set_error(SMI_E_ARG, "ppo epochs: act_dim in [1,32]");
  const int64_t lds = fused_lds_bytes(a.B, a.obs_dim, a.h1, a.h2, a.act_dim, a.critic_h1,
                                      a.critic_h2);
  if (lds > 160 * 1024) return set_error(SMI_E_NOFIT, "ppo epochs: parameters do not fit LDS");
  *lds_out = lds;
  return SMI_OK;
}

int launch_ppo_fused(const smi_ppo_args* args, hipStream_t stream) {
  int64_t lds = 0;
  int rc = fused_check(*args, &lds);
  if (rc) return rc;
  if (args->B < 2 && !args->adv_moments)
    return set_error(SMI_E_ARG, "ppo_fused: B >= 2 needed for the unbiased advantage std");
  const MlpLayout LA = mlp_layout(args->obs_dim, args->h1, args->h2, args->act_dim, 1);
  const MlpLayout LC = mlp_layout(args->obs_dim, args->critic_h1, args->critic_h2, 1, 0);
  if (LA.fcount > kFWG * kAdamPer || LC.fcount > kFWG * kAdamPer)
    return set_error(SMI_E_NOFIT, "ppo_fused: network larger than smi_ppo_fused_max_params()");
  allow_lds(ppo_fused_kernel, (size_t)lds);
  hipLaunchKernelGGL(ppo_fused_kernel, dim3(2), dim3(kFWG), (size_t)lds, stream, *args);
  return check_launch("ppo_fused_kernel");
}

int64_t ppo_fused_max_params() { return (int64_t)kFWG * kAdamPer; }

int64_t ppo_xbuf_floats(int D, int H1, int H2, int A, int cH1, int cH2, int mode) {
  return x_layout(D, H1, H2, A, cH1, cH2, mode).total;
}

int launch_ppo_epoch_grad(const smi_ppo_args* args, int epoch, hipStream_t stream) {
  int64_t lds = 0;
  int rc = fused_check(*args, &lds);
  if (rc) return rc;
  if (!args->xbuf || !args->dp_state || !args->adv_moments)
    return set_error(SMI_E_ARG, "ppo_epoch_grad: xbuf, dp_state and adv_moments are required");
  allow_lds(ppo_epoch_grad_kernel, (size_t)lds);
  hipLaunchKernelGGL(ppo_epoch_grad_kernel, dim3(2), dim3(kFWG), (size_t)lds, stream, *args, epoch);
  return check_launch("ppo_epoch_grad_kernel");
}

int launch_ppo_epoch_apply(const smi_ppo_args* args, int epoch, hipStream_t stream) {
  if (!args->xbuf || !args->dp_state)
    return set_error(SMI_E_ARG, "ppo_epoch_apply: xbuf and dp_state are required");
  hipLaunchKernelGGL(ppo_epoch_apply_kernel, dim3(1), dim3(kWG), 0, stream, *args, epoch);
  return check_launch("ppo_epoch_apply_kernel");
}

}  // namespace smi

#ifdef SMI_PROF
// Developer hook (SMI_PROF builds only): copy out and clear the phase ticks.
extern "C" int smi_phase_ticks(unsigned long long* out /* [64] */) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(smi::g_phase_ticks), sizeof(smi::g_phase_ticks)) != hipSuccess)
    return SMI_E_LAUNCH;
  static const unsigned long long zero[64] = {};
  return hipMemcpyToSymbol(HIP_SYMBOL(smi::g_phase_ticks), zero, sizeof(zero)) == hipSuccess ? SMI_OK : SMI_E_LAUNCH;
}
#endif
