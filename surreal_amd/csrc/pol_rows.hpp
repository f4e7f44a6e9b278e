// pol_rows.hpp — the per-row pieces of the PPO policy loss (ppo.py:203-224,
// 262-284, 553-575; ppo_net.py:29-72) shared by the row kernels of
// ppo_rnn.hip and the policy-gradient prologue of the fused head input-gradient
// chain (head_kernels.hip): the packed row layout, the argument blocks, the
// DiagGauss row terms and the epoch's early-stop / adapt-coefficient decision.
#pragma once
#include "smi_device.hpp"
#include "smi_internal.hpp"

namespace smi {

// policy sums (pstat, double): one forward over the E*B training rows
enum {
  PS_KL = 0,       // sum KL(ref || learn)                       ppo.py:265,553
  PS_SURR,         // clip: sum -ratio*adv; adapt: sum adv*lik/clamp(lik_b)
  PS_CLIP,         // clip: sum max(surr, clipped surr)          ppo.py:213
  PS_ISW,          // sum lik / (lik_b + 1e-4)                   ppo.py:573
  PS_BL,           // sum lik_b                                  ppo.py:572
  PS_RBD,          // sum KL(ref || behave)                      ppo.py:574
  PS_RET,          // sum returns                                ppo.py:570
  PS_N = 8
};
// device control block (int / float scratch)
enum { CI_STOP = 0, CI_RUNS, CI_NG, CI_NP, CI_COUNT = 8 };
enum { CF_KLCOEF = 0, CF_SURRW, CF_COUNT = 8 };

// fields of a packed row: A actions, 2A behaviour parameters, the advantage,
// then the row's behaviour-policy terms, fixed for the whole learn() (the
// behaviour parameters and the reference policy do not change across epochs):
// the clamped behaviour likelihood and the row's KL(ref || behaviour) term,
// computed once by row_pack_kernel instead of in every epoch's row passes
__host__ __device__ inline int row_w(int A) { return 3 * A + 3; }
__host__ __device__ inline int rin_adv(int A) { return 3 * A; }
__host__ __device__ inline int rin_bl(int A) { return 3 * A + 1; }
__host__ __device__ inline int rin_rbd(int A) { return 3 * A + 2; }
// rowin is blocked by 64 rows: block b holds field f of rows 64b .. 64b + 63
// as 64 consecutive floats, the block's fields back to back, so one wave's
// row loads read one contiguous ~5 KB run (a field-major [W][NE] layout made
// every wave touch W DRAM pages per row batch)
__host__ __device__ inline int64_t rin_idx(int W, int64_t n, int f) {
  return (n >> 6) * ((int64_t)W << 6) + ((int64_t)f << 6) + (n & 63);
}

struct DecideArgs {
  const double* ps; int e, Ep, mode; double kl_target; float eta; int64_t N;
  const float* hyper; const float* lv; int A; float c_ent;
  int* ci; float* cf; float* stats;
};

struct PolRowArgs {
  int B, T, E, A, mode;
  const float* mu;        // [NE][A] learner means (tanh applied)
  const float* lv;        // [A] learner log_var
  const float* refmu;     // [NE][A]
  const float* ref_lv;    // [A]
  const float* actions;   // [B][T][A]
  const float* behave;    // [B][T][2A]
  const float* adv;       // [B][E] raw
  const float* ret;       // [B][E]
  const float* rowin;     // {actions | behave | raw adv | bl | rbd} blocked by 64 rows (rin_idx)
  const float* ret_tm;    // [NE] time-major returns
  const double* moments;  // [3] global (sum, sumsq, n) of adv, or null (no norm)
  int norm_adv;
  float c_ll;
  const float* hyper;
  const int* skip;
  // outputs
  double* part;           // [nblk][PS_N]
  float* dz;              // [NE][A]   (grad pass)
  float* lvpart;          // [nblk][A] (grad pass)
  const float* cf;        // device coefficients (grad pass)
  float invN;
  // grad pass, single rank: the statistics pass's partials ([dec_nb][PS_N]) and
  // the decision's arguments; each block reduces them itself (the order of
  // reduce_decide_kernel) and decides, block 0 writes the decision's outputs
  // (one launch fewer per epoch than reduce_decide_kernel + this pass)
  const double* dec_part; int dec_nb;
  DecideArgs dec;
};

// ppo.py:402-405: (adv - mean) / max(std, 1e-4), std unbiased over all B*E;
// the fp64 moments are turned into (mean_f, max(std_f, 1e-4)) once per thread
// (AdvNorm), outside the row loops: per row only the fp32 subtract and divide
struct AdvNorm {
  bool on; float mean, den;
  __device__ explicit AdvNorm(const PolRowArgs& a) : on(a.norm_adv && a.moments), mean(0.f), den(1.f) {
    if (on) init(a.moments[0], a.moments[1], a.moments[2]);
  }
  // from moments already in registers (PolGradPre)
  __device__ AdvNorm(const PolRowArgs& a, const double* mom) : on(a.norm_adv && a.moments), mean(0.f), den(1.f) {
    if (on) init(mom[0], mom[1], mom[2]);
  }
  __device__ void init(double s, double ss, double n) {
    const double m = s / n;
    const double var = (ss - n * m * m) / (n - 1.0);
    mean = (float)m;
    den = fmaxf((float)sqrt(var > 0.0 ? var : 0.0), 1e-4f);
  }
  __device__ float operator()(float raw) const { return on ? (raw - mean) / den : raw; }
};

// Row access of the per-row loss kernels.  AT > 0: the action width is a
// compile-time constant (the benched A = 8 and HalfCheetah's 6), so a row's
// values live in registers (fully unrolled loops) and rows of 4k floats move
// as float4 (16-byte aligned: row offsets are multiples of 4A bytes); AT == 0:
// any A <= 32 through runtime loops.
template <int AT>
__device__ __forceinline__ void ld_row(float* dst, const float* __restrict__ src, int A) {
  if constexpr (AT > 0 && AT % 4 == 0) {
#pragma unroll
    for (int q = 0; q < AT / 4; ++q) {
      const float4 v = reinterpret_cast<const float4*>(src)[q];
      dst[4 * q] = v.x; dst[4 * q + 1] = v.y; dst[4 * q + 2] = v.z; dst[4 * q + 3] = v.w;
    }
  } else if constexpr (AT > 0) {
#pragma unroll
    for (int j = 0; j < AT; ++j) dst[j] = src[j];
  } else {
    for (int j = 0; j < A; ++j) dst[j] = src[j];
  }
}
template <int AT>
__device__ __forceinline__ void st_row(float* __restrict__ dst, const float* src, int A) {
  if constexpr (AT > 0 && AT % 4 == 0) {
#pragma unroll
    for (int q = 0; q < AT / 4; ++q)
      reinterpret_cast<float4*>(dst)[q] = float4{src[4 * q], src[4 * q + 1], src[4 * q + 2], src[4 * q + 3]};
  } else if constexpr (AT > 0) {
#pragma unroll
    for (int j = 0; j < AT; ++j) dst[j] = src[j];
  } else {
    for (int j = 0; j < A; ++j) dst[j] = src[j];
  }
}
template <int AT>
__device__ __forceinline__ float row_loglik(const float* act, const float* mu, const float* sd,
                                            const float* logsd, int A, float c_ll) {
  float s = 0.f, l = 0.f;
#pragma unroll
  for (int j = 0; j < (AT > 0 ? AT : A); ++j) {
    const float u = (act[j] - mu[j]) / sd[j];
    s += u * u;
    l += logsd[j];
  }
  return (-0.5f * s - c_ll) - l;
}
template <int AT>
__device__ __forceinline__ float row_kl(const float* mu0, const float* sd0, const float* mu1,
                                        const float* sd1, int A) {
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int j = 0; j < (AT > 0 ? AT : A); ++j) {
    s1 += logf(sd1[j] / sd0[j]);
    const float d = mu0[j] - mu1[j];
    s2 += (sd0[j] * sd0[j] + d * d) / (2.f * (sd1[j] * sd1[j]));
  }
  return (s1 + s2) - 0.5f * (float)(AT > 0 ? AT : A);
}

// row_loglik with the std's reciprocal: (a - mu) * (1 / sd) instead of the
// IEEE divide (one rounding more, within the parity envelope): the learner's
// std is a per-column constant (reciprocal hoisted out of the row loop), the
// behaviour policy's is per row (one IEEE-rounded 1.f / sd per row element,
// shared by every term of the row that divides by it; not the approximate
// v_rcp_f32, whose ~1 ulp error and denormal flush the learner-std path does
// not have either)
template <int AT>
__device__ __forceinline__ float row_loglik_r(const float* act, const float* mu, const float* isd,
                                              const float* logsd, int A, float c_ll) {
  float s = 0.f, l = 0.f;
#pragma unroll
  for (int j = 0; j < (AT > 0 ? AT : A); ++j) {
    const float u = (act[j] - mu[j]) * isd[j];
    s += u * u;
    l += logsd[j];
  }
  return (-0.5f * s - c_ll) - l;
}

// row_kl with BOTH distributions' stds fixed per column (the reference policy
// against the learner: log(sd1 / sd0), sd0^2 and 2 sd1^2 are hoisted out of the
// row loop as lkl, s02, den2 — the same operations in the same order, computed
// once per workgroup instead of once per row)
template <int AT>
__device__ __forceinline__ float row_kl_cc(const float* mu0, const float* mu1, const float* lkl,
                                           const float* s02, const float* iden2, int A) {
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int j = 0; j < (AT > 0 ? AT : A); ++j) {
    s1 += lkl[j];
    const float d = mu0[j] - mu1[j];
    s2 += (s02[j] + d * d) * iden2[j];
  }
  return (s1 + s2) - 0.5f * (float)(AT > 0 ? AT : A);
}

// KL(reference || behaviour) of a row: the reference std per column (its
// log and square hoisted), the behaviour std per row through its log (already
// formed for the log-likelihood) and reciprocal
template <int AT>
__device__ __forceinline__ float row_kl_rb(const float* mu0, const float* lsd0, const float* s02,
                                           const float* mu1, const float* lsd1, const float* isd1,
                                           int A) {
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int j = 0; j < (AT > 0 ? AT : A); ++j) {
    s1 += lsd1[j] - lsd0[j];
    const float d = mu0[j] - mu1[j];
    s2 += (s02[j] + d * d) * (0.5f * (isd1[j] * isd1[j]));
  }
  return (s1 + s2) - 0.5f * (float)(AT > 0 ? AT : A);
}

// field j .. j + AT - 1 of row n from the blocked rowin
template <int AT>
__device__ __forceinline__ void ld_fields(float* dst, const float* __restrict__ rowin, int64_t /*N*/,
                                          int64_t n, int f0, int A) {
  const int W = row_w(AT > 0 ? AT : A);
#pragma unroll
  for (int j = 0; j < (AT > 0 ? AT : A); ++j) dst[j] = rowin[rin_idx(W, n, f0 + j)];
}

// a row's behaviour-policy terms (row_pack_kernel, once per learn): the
// clamped behaviour likelihood max(exp(loglik(ac; bmu, bsd)), 1e-5) and the
// KL(ref || behaviour) row term (ppo.py:203-224's prob_behave, 569's
// ref_behave_diff), the ops of the row passes that computed them per epoch
template <int AT>
__device__ __forceinline__ void behave_terms(const float* ac, const float* bmu, const float* bsd,
                                             const float* rm, const float* lrsig, const float* s02,
                                             int A, float c_ll, float& bl, float& rbd) {
  constexpr int AM = AT > 0 ? AT : 32;
  float blsd[AM], ibsd[AM];
#pragma unroll
  for (int j = 0; j < (AT > 0 ? AT : A); ++j) {
    blsd[j] = logf(bsd[j]);
    ibsd[j] = 1.f / bsd[j];
  }
  bl = fmaxf(expf(row_loglik_r<AT>(ac, bmu, ibsd, blsd, A, c_ll)), 1e-5f);
  rbd = row_kl_rb<AT>(rm, lrsig, s02, bmu, blsd, ibsd, A);
}

// After the (all-reduced) policy sums of POLICY_FWD(e): early stop, adapt
// coefficient and statistics (ppo.py:265-284, 541-557, 568-575).  ps = the
// sums; write = store the decision (stats, stop flag, coefficients), else only
// return it (the blocks of a fused gradient pass other than block 0)
struct Decision { int stop; float surrw, klcoef; };
// pre (the gradient pass): the stop flag and beta loaded at the pass's start,
// and log(exp(lv)) per column from its LDS (the same ops as the entropy's)
struct DecidePre { int stop; float beta; const float* lsig; };
__device__ inline Decision policy_decide_body(const DecideArgs& a, const double* ps, bool write,
                                              const DecidePre* pre = nullptr) {
  Decision r{1, 0.f, 0.f};
  if (pre ? pre->stop : a.ci[CI_STOP]) return r;
  const double n = (double)a.N;
  const float kl = (float)(ps[PS_KL] / n);
  // statistics of the forward with the current parameters (curr_pol after the
  // previous update, or ref/behave terms before any)
  if (write) {
    a.stats[SMI_ST_AVG_IS_WEIGHT] = (float)(ps[PS_ISW] / n);
    a.stats[SMI_ST_AVG_BEHAVE_LIK] = (float)(ps[PS_BL] / n);
    a.stats[SMI_ST_REF_BEHAVE_DIFF] = (float)(ps[PS_RBD] / n);
    a.stats[SMI_ST_AVG_RETURN] = (float)(ps[PS_RET] / n);
  }
  if (a.e >= 1) {
    if (write) a.stats[SMI_ST_POL_KL] = kl;                 // ppo.py:555
    if ((double)kl > a.kl_target * 4.0) {                    // ppo.py:556
      if (write) a.ci[CI_STOP] = 1;
      return r;
    }
  }
  if (a.e >= a.Ep) {
    if (write) a.ci[CI_STOP] = 1;                            // loop finished
    return r;
  }
  r.stop = 0;
  // loss statistics of update e
  r.surrw = (float)(1.0 / n);
  if (write) {
    float ent = 0.f;
    for (int j = 0; j < a.A; ++j) ent += pre ? pre->lsig[j] : logf(expf(a.lv[j]));
    ent = 0.5f * ent + a.c_ent;
    a.stats[SMI_ST_ENTROPY] = ent;
    a.cf[CF_SURRW] = r.surrw;
  }
  if (a.mode == 0) {
    if (write) {
      a.stats[SMI_ST_SURR_LOSS] = (float)(ps[PS_SURR] / n);
      a.stats[SMI_ST_CLIP_SURR_LOSS] = (float)(ps[PS_CLIP] / n);
      a.cf[CF_KLCOEF] = 0.f;
    }
  } else {
    const float beta = pre ? pre->beta : a.hyper[SMI_HYP_BETA];
    const float surr = -(float)(ps[PS_SURR] / n);
    float loss = surr + beta * kl;
    float coef = beta;
    if ((double)kl - 2.0 * a.kl_target > 0.0) {              // ppo.py:275
      const float d = kl - (float)(2.0 * a.kl_target);
      loss += a.eta * (d * d);
      coef += 2.f * a.eta * d;
    }
    r.klcoef = (float)(coef / n);
    if (write) {
      a.stats[SMI_ST_SURR_LOSS] = surr;
      a.stats[SMI_ST_KL_LOSS_ADAPT] = loss;
      a.stats[SMI_ST_POL_KL_ADAPT] = kl;
      a.stats[SMI_ST_POL_KL] = kl;
      a.cf[CF_KLCOEF] = r.klcoef;
    }
  }
  return r;
}


// ---- the gradient row pass (policy_rows_grad_kernel; the fused head chain's
// prologue, head_kernels.hip) ----
// LDS of the pass: the stds of both policies and the decision's sums
struct PolGradShared { float sig[32], lsig[32], rsig[32]; double sps[PS_N]; };

// the epoch's loss weights: the surrogate weight (1/N) and the KL weight
// (adapt: (beta + 2 eta relu(kl - 2kt)) / N; clip: 0), from cf, or, with
// a.dec_part (one rank), decided here from the statistics pass's partials
// (reduced in reduce_decide_kernel's order: lane i sums blocks i, i + 64, ...
// then the wave butterfly, so every workgroup reaches the same decision; block
// 0 writes it).  Also stages the stds in sh.  Returns true when the epoch does
// not train (early stop / loop done) or skip[0] != 0 (the caller's skip
// flag, optional): the caller returns, uniformly.  Every
// thread of the workgroup must call it (it has barriers).
//
// Every global value the pass reads before its rows — the stds' log_vars, the
// decision's flag and beta, the clip range, the advantage moments, the
// coefficients and the partials — is loaded up front, together (PolGradPre;
// the partials CH 64-block slabs per round trip): read where used, each was a
// dependent memory round trip of its own (a load the compiler cannot move
// above the decision's global stores, or a per-lane-conditional load sunk into
// its branch), ~12 of them at C3's 336 partials.  The sums are the same adds
// in the same order (lane i: blocks i, i + 64, ...).
// (a global, never written: a constant-space zero made the pointer selects
// below flat loads, whose lgkmcnt waits held back the partials' loads)
static __device__ double g_pol_zero[4];
struct PolGradPre {
  int stop; float beta, clip_lo, clip_hi, cf_surrw, cf_klcoef; double mom[3];
};
template <int CH = 4>
__device__ inline bool pol_grad_weights(const PolRowArgs& a, PolGradShared& sh, float& wsurr,
                                        float& wkl, PolGradPre& pre, const int* skip = nullptr) {
  const int A = a.A;
  const bool dec = a.dec_part != nullptr;
  const int lane = threadIdx.x & 63;
  const bool dw = dec && threadIdx.x < 64;      // wave 0 reduces the partials
  const int nb = a.dec_nb;
  const double2* P = reinterpret_cast<const double2*>(a.dec_part);
  // vector loads first: the stds' inputs (column threadIdx.x, A <= 32 <
  // blockDim.x, clamped) and the first CH slabs of partials (clamped) ...
  const int jc = min((int)threadIdx.x, A - 1);
  float lvj = a.lv[jc], rlvj = a.ref_lv[jc];
  double2 v[CH][PS_N / 2];
  auto load_slabs = [&](int i0) {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int64_t ic = min(i0 + 64 * c + lane, nb - 1);
#pragma unroll
      for (int q = 0; q < PS_N / 2; ++q) v[c][q] = P[ic * (PS_N / 2) + q];
    }
  };
  if (dw) load_slabs(0);
  // ... then the scalars (their lgkmcnt wait ahead of the slab loads was a
  // round trip of its own), the caller's skip flag among them
  const float* fz = reinterpret_cast<const float*>(g_pol_zero);
  const int* zi = reinterpret_cast<const int*>(g_pol_zero);
  int sk;
  {
    const int* cip = dec ? a.dec.ci + CI_STOP : zi;
    const float* bp = dec ? a.dec.hyper + SMI_HYP_BETA : fz;
    const float* cfp = dec ? fz : a.cf;
    const double* mp = (a.norm_adv && a.moments) ? a.moments : g_pol_zero;
    sk = *(skip ? skip : zi);
    pre.stop = *cip;
    pre.beta = *bp;
    pre.clip_lo = a.hyper[SMI_HYPX_CLIP_LO];
    pre.clip_hi = a.hyper[SMI_HYPX_CLIP_HI];
    pre.cf_surrw = cfp[CF_SURRW];
    pre.cf_klcoef = cfp[CF_KLCOEF];
    pre.mom[0] = mp[0]; pre.mom[1] = mp[1]; pre.mom[2] = mp[2];
  }
  double t[PS_N];
#pragma unroll
  for (int j = 0; j < PS_N; ++j) t[j] = 0.0;
  if (dw) {
    // the slabs pinned (else the last one's loads sank into its per-lane
    // branch), then the guarded adds; further slab groups (> 64 CH partials)
    // one round trip each
    auto add_slabs = [&](int i0) {
#pragma unroll
      for (int c = 0; c < CH; ++c)
#pragma unroll
        for (int q = 0; q < PS_N / 2; ++q) asm volatile("" : "+v"(v[c][q].x), "+v"(v[c][q].y));
#pragma unroll
      for (int c = 0; c < CH; ++c) {
        if (i0 + 64 * c + lane < nb) {
#pragma unroll
          for (int q = 0; q < PS_N / 2; ++q) { t[2 * q] += v[c][q].x; t[2 * q + 1] += v[c][q].y; }
        }
      }
    };
    add_slabs(0);
    for (int i0 = 64 * CH; i0 < nb; i0 += 64 * CH) { load_slabs(i0); add_slabs(i0); }
  }
  if (sk != 0) return true;      // uniform: before the first barrier
  asm volatile("" : "+v"(lvj));
  asm volatile("" : "+v"(rlvj));
  if ((int)threadIdx.x < A) {
    const int j = threadIdx.x;
    sh.sig[j] = expf(lvj);
    sh.lsig[j] = logf(sh.sig[j]);
    sh.rsig[j] = expf(rlvj);
  }
  if (dec) {
    if (threadIdx.x < 64) {
#pragma unroll
      for (int j = 0; j < PS_N; ++j) {
        const double u = wave_sum_d(t[j]);
        if (lane == 0) sh.sps[j] = u;
      }
    }
    __syncthreads();
    const bool wr = blockIdx.x == 0 && threadIdx.x == 0;
    if (wr) {
      double* out = const_cast<double*>(a.dec.ps);
      for (int j = 0; j < PS_N; ++j) out[j] = sh.sps[j];
    }
    const DecidePre dp{pre.stop, pre.beta, sh.lsig};
    const Decision dd = policy_decide_body(a.dec, sh.sps, wr, &dp);
    wsurr = dd.surrw;
    wkl = dd.klcoef;
    return dd.stop != 0;
  }
  __syncthreads();
  wsurr = pre.cf_surrw;
  wkl = pre.cf_klcoef;
  return false;
}

// per-column factors of the row pass, hoisted; divisions by them become
// multiplications by their reciprocals (as in policy_rows_stats_kernel)
template <int AT>
struct PolGradCols {
  static constexpr int AM = AT > 0 ? AT : 32;
  float lsig[AM], inv1[AM], is1sq[AM], is1cu[AM], rs2[AM];
  float clip_lo, clip_hi;
  int A;
  __device__ PolGradCols(const PolGradPre& pre, const PolGradShared& sh, int A_) : A(A_) {
#pragma unroll
    for (int j = 0; j < (AT > 0 ? AT : A_); ++j) {
      const float sg = sh.sig[j], rsig = sh.rsig[j];
      lsig[j] = sh.lsig[j];
      inv1[j] = 1.f / sg;
      is1sq[j] = 1.f / (sg * sg);
      is1cu[j] = 1.f / (sg * sg * sg);
      rs2[j] = rsig * rsig;
    }
    clip_lo = pre.clip_lo;
    clip_hi = pre.clip_hi;
  }
};

// one row's inputs of the gradient pass (loaded before the epoch's weights
// are known: their latency overlaps the decision)
template <int AT>
struct PolGradRow {
  static constexpr int AM = AT > 0 ? AT : 32;
  float m[AM], rm[AM], ac[AM], adv, bl;
  __device__ void load(const PolRowArgs& a, int64_t n, int A) {
    const int64_t N = (int64_t)a.E * a.B;
    ld_row<AT>(m, a.mu + n * A, A);
    ld_row<AT>(rm, a.refmu + n * A, A);
    ld_fields<AT>(ac, a.rowin, N, n, 0, A);
    adv = a.rowin[rin_idx(row_w(A), n, rin_adv(A))];
    bl = a.rowin[rin_idx(row_w(A), n, rin_bl(A))];
  }
};

// a loaded row's dz (gradient at the tanh pre-activation) and its d/dstd
// terms added into glv
template <int AT>
__device__ __forceinline__ void pol_grad_compute(const PolRowArgs& a, const PolGradCols<AT>& c,
                                                 const AdvNorm& nadv, const PolGradRow<AT>& x,
                                                 float wsurr, float wkl, float* dz, float* glv) {
  constexpr int AM = AT > 0 ? AT : 32;
  const int A = c.A;
  const float* m = x.m;
  const float* rm = x.rm;
  const float* ac = x.ac;
  const float av = nadv(x.adv);
  const float ll = row_loglik_r<AT>(ac, m, c.inv1, c.lsig, A, a.c_ll);
  const float ex = expf(ll);
  const float lp = fmaxf(ex, 1e-5f);
  const float bl = x.bl;
  float g_lp;
  if (a.mode == 0) {
    const float ratio = lp / bl;
    const float cr = fminf(fmaxf(ratio, c.clip_lo), c.clip_hi);
    const float surr = -ratio * av, csur = -cr * av;
    // max() routes to the unclipped term unless the clipped one is strictly
    // larger (then the ratio is outside the clamp and the gradient is 0)
    g_lp = ((surr >= csur) ? -(wsurr * av) : 0.f) / bl;
  } else {
    g_lp = (-wsurr * av) / fmaxf(bl, 1e-2f);
  }
  const float g_ll = (ex >= 1e-5f) ? g_lp * ex : 0.f;    // clamp + exp backward
#pragma unroll
  for (int j = 0; j < (AT > 0 ? AT : A); ++j) {
    const float i1 = c.inv1[j];
    const float u = (ac[j] - m[j]) * i1;
    float gmu = g_ll * (u * i1);
    float gsd = g_ll * (u * u * i1 - i1);
    if (wkl != 0.f) {
      const float d = rm[j] - m[j];
      gmu += wkl * (-d * c.is1sq[j]);
      gsd += wkl * (i1 - (c.rs2[j] + d * d) * c.is1cu[j]);
    }
    glv[j] += gsd;
    dz[j] = gmu * (1.f - m[j] * m[j]);                    // tanh backward
  }
}

// row n's dz and d/dstd terms (load + compute)
template <int AT>
__device__ __forceinline__ void pol_grad_row(const PolRowArgs& a, const PolGradCols<AT>& c,
                                             const AdvNorm& nadv, int64_t n, float wsurr, float wkl,
                                             float* dz, float* glv) {
  PolGradRow<AT> x;
  x.load(a, n, c.A);
  pol_grad_compute<AT>(a, c, nadv, x, wsurr, wkl, dz, glv);
}

// ---- the statistics row pass (policy_rows_stats_kernel, adapt mode; the
// fused head forward's epilogue) ----
// per-column terms of the learner std (log-likelihood, KL(ref || learner))
// and the reference std (KL(ref || behaviour)), hoisted out of the row loop
template <int AT>
struct PolStatsCols {
  static constexpr int AM = AT > 0 ? AT : 32;
  float isig[AM], lsig[AM], lkl[AM], s02[AM], iden2[AM], lrsig[AM];
  int A;
  // sig / lsig / rsig: exp(lv), log(exp(lv)), exp(ref_lv) per column
  __device__ PolStatsCols(const float* sig, const float* lsg, const float* rsg, int A_) : A(A_) {
#pragma unroll
    for (int j = 0; j < (AT > 0 ? AT : A_); ++j) {
      const float sg = sig[j], rsig = rsg[j];
      lsig[j] = lsg[j];
      isig[j] = 1.f / sg;
      lkl[j] = logf(sg / rsig);                // row_kl(rm, rsig, m, sig)'s per-column terms
      s02[j] = rsig * rsig;
      iden2[j] = 1.f / (2.f * (sg * sg));
      lrsig[j] = logf(rsig);
    }
  }
};

// adapt-mode sums of one row into acc[PS_N] (policy_rows_stats_kernel's row
// pass, FUSE off: the same ops in the same order); m = the row's learner means
// the same per-column terms held in LDS (policy_rows_stats_lean_kernel: the
// row pass's registers left to more waves in flight)
struct PolStatsColsLds {
  float isig[32], lsig[32], lkl[32], s02[32], iden2[32], lrsig[32];
  int A;
};
__device__ inline void pol_stats_cols_fill(PolStatsColsLds& c, const float* lv, const float* ref_lv,
                                           int A) {
  for (int j = threadIdx.x; j < A; j += blockDim.x) {
    const float sg = expf(lv[j]), rsig = expf(ref_lv[j]);
    c.lsig[j] = logf(sg);
    c.isig[j] = 1.f / sg;
    c.lkl[j] = logf(sg / rsig);
    c.s02[j] = rsig * rsig;
    c.iden2[j] = 1.f / (2.f * (sg * sg));
    c.lrsig[j] = logf(rsig);
  }
  if (threadIdx.x == 0) c.A = A;
}

template <int AT, class Cols>
__device__ __forceinline__ void pol_stats_row_adapt(const PolRowArgs& a, const Cols& c,
                                                    const AdvNorm& nadv, const float* m,
                                                    const float* rm, const float* ac,
                                                    float bl, float rbd, float adv,
                                                    float ret, double* acc) {
  const int A = c.A;
  const float av = nadv(adv);
  const float ex = expf(row_loglik_r<AT>(ac, m, c.isig, c.lsig, A, a.c_ll));
  const float lp = fmaxf(ex, 1e-5f);
  acc[PS_KL] += (double)row_kl_cc<AT>(rm, m, c.lkl, c.s02, c.iden2, A);
  acc[PS_SURR] += (double)(av * (lp / fmaxf(bl, 1e-2f)));
  acc[PS_CLIP] += 0.0;
  acc[PS_ISW] += (double)(lp / (bl + 1e-4f));
  acc[PS_BL] += (double)bl;
  acc[PS_RBD] += (double)rbd;
  acc[PS_RET] += (double)ret;
}

}  // namespace smi
