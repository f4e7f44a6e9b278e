// capi.hip — the extern "C" boundary declared in include/surreal_mi.h.
// Validates arguments, forwards to the launchers, and keeps the thread-local
// error message for smi_last_error().
#include <stdio.h>
#include <string.h>
#include <atomic>
#include "smi_device.hpp"
#include "smi_internal.hpp"

namespace smi {

static thread_local char g_err[512] = "";

int set_error(int code, const char* msg) {
  snprintf(g_err, sizeof(g_err), "%s", msg);
  return code;
}

int check_launch(const char* what) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    snprintf(g_err, sizeof(g_err), "%s: %s", what, hipGetErrorString(e));
    return -(int)e;
  }
  return SMI_OK;
}

// ------------------------------------------------------------ kernel timing
// process-wide record (measurement only): slots are claimed atomically, so
// launches from several threads may record at once
static bool g_kt = false;
static const int kKtCap = 16384;
static hipEvent_t* g_kt_ev = nullptr;        // [2 * kKtCap]
static std::atomic<int> g_kt_n{0};
struct KtRec { int cls; double flops; };
static KtRec g_kt_rec[kKtCap];

bool ktime_on() { return g_kt; }
int ktime_begin(hipStream_t st) {
  if (!g_kt) return -1;
  const int slot = g_kt_n.fetch_add(1);
  if (slot >= kKtCap) return -1;
  (void)hipEventRecord(g_kt_ev[2 * slot], st);
  return slot;
}
void ktime_end(int slot, int cls, double flops, hipStream_t st) {
  if (slot < 0) return;
  g_kt_rec[slot].cls = cls;
  g_kt_rec[slot].flops = flops;
  (void)hipEventRecord(g_kt_ev[2 * slot + 1], st);
}

// ---------------------------------------------------------- workspace contexts
// A context = one caller-owned device workspace.  The calling thread's current
// context (smi_context_make_current) serves every workspace request of the
// launches that thread enqueues; without one, the default context
// (smi_set_workspace) does.
// A destroyed context is only marked dead, never freed: another thread may
// still hold it as its current context (a thread_local this thread cannot
// clear), and then falls back to the default context instead of reading freed
// memory.  A context is 24 bytes; the workspace itself belongs to the caller.
}  // namespace smi
struct smi_context { void* ws; int64_t bytes; std::atomic<bool> alive; };
namespace smi {
static smi_context g_default_ctx{nullptr, 0, {true}};
#ifdef SMI_FAULT_INJECTION
static int g_fault = SMI_FAULT_NONE;
int fault() { return g_fault; }
#endif
static thread_local smi_context* t_ctx = nullptr;
static smi_context* cur_ctx() {
  smi_context* c = t_ctx;
  return c && c->alive.load(std::memory_order_acquire) ? c : &g_default_ctx;
}
// floats at the start of the current workspace that hold partials a later
// launch of this thread still reads (the BPTT + heads' dW launch's split-K
// partials until its group's reducer): every request is served above them
static thread_local int64_t t_ws_reserved = 0;
void workspace_reserve(int64_t nfloats) { t_ws_reserved = nfloats > 0 ? nfloats : 0; }
int64_t smi_workspace_floats() {
  const smi_context* c = cur_ctx();
  return c->ws ? c->bytes / 4 - t_ws_reserved : 0;
}
float* workspace_f32(int64_t nfloats) {
  const smi_context* c = cur_ctx();
  if (!c->ws || nfloats + t_ws_reserved > c->bytes / 4) return nullptr;
  return static_cast<float*>(c->ws) + t_ws_reserved;
}

// declared in the other translation units
int launch_zfilter_apply(const float*, float*, int64_t, int, const float*, const float*,
                         const float*, float, hipStream_t);
int launch_colstats(const float*, int64_t, int, int64_t, int, float*, float*, float*,
                    hipStream_t);
int launch_reward_filter(float*, int64_t, float, int, float*, float*, float*, float, double*,
                         hipStream_t);
int launch_reward_filter_commit(const double*, float*, float*, float*, hipStream_t);
int launch_layernorm_fwd(const float*, int64_t, int64_t, int, const float*, const float*, float,
                         float*, int64_t, float*, float*, hipStream_t);
int launch_layernorm_bwd(const float*, int64_t, const float*, int64_t, const float*, const float*,
                         const float*, int64_t, int, int, float*, int64_t, float*, float*,
                         hipStream_t);
int launch_diag_gauss(const float*, const float*, const float*, int64_t, int, float*, float*,
                      float*, float*, hipStream_t);
int launch_mlp_forward(const float*, int, int, int, int, int, int, const float*, int64_t,
                       int64_t, int, const float*, const float*, const float*, float, float*,
                       hipStream_t);
int launch_moments(const float*, int64_t, const double*, int, double*, hipStream_t);
int launch_zfilter_tmajor(const float*, const float*, int, int, int, int, int, const float*,
                          const float*, const float*, float, float*, int, int, hipStream_t);
int launch_adam_clip(float*, const float*, float*, float*, int64_t, int*, const float*, float,
                     float, float, float, float, float, const int*, float*, hipStream_t);
int launch_mse_grad(const float*, int64_t, const float*, int64_t, float*, float*, hipStream_t);
int launch_neg_mean_grad(const float*, int64_t, int64_t, float*, float*, hipStream_t);
int launch_tanh_backward(const float*, int64_t, const float*, int64_t, int64_t, int, float*,
                         int64_t, hipStream_t);
int launch_copy_cols(const float*, int64_t, int64_t, int, float*, int64_t, hipStream_t);
int launch_linear_fwd_cat(const float*, int64_t, int, int, const float*, int64_t, const float*, int,
                          int, float*, int64_t, const float*, int64_t, int, hipStream_t);
int launch_soft_update(float*, const float*, int64_t, float, hipStream_t);
int launch_copy_bytes16(const void*, void*, int64_t, hipStream_t);
int launch_copy_gather(void*, const void* const*, const int64_t*, const int64_t*, int, hipStream_t);
bool head_fused_ok(int in, int64_t ldx, int h1, int h2, int out, const float* X,
                   const float* W1, const float* W2, const float* W3);
struct PolRowArgs;
int launch_mlp3_stacked(const float* P, int64_t pstride, const int64_t* o6, int in, int h1, int h2,
                        int out, int act_out, const float* x, int64_t ldx, int n, float* y,
                        int64_t ldy, hipStream_t st);
int launch_head_fwd_fused(const float* X, int64_t ldx, int64_t rows, int in, const float* W1,
                          const float* b1, int h1, const float* W2, const float* b2, int h2,
                          const float* W3, const float* b3, int out, int tanh_out, float* HA1,
                          float* HA2, float* Y, int64_t ldy, float* W1T, float* W2T,
                          hipStream_t st, const int* skip, const float* vret = nullptr,
                          float* vgrad = nullptr, float vscale = 0.f,
                          const PolRowArgs* ps = nullptr, double* vpart = nullptr);
bool head_fwd_ps_ok(int h1, int h2, int out);
int launch_head_bwd_fused(const float* dZ, int out, int64_t rows, const float* W3,
                          const float* W2T, const float* W1T, int h1, int h2, int dx0, int dxn,
                          const float* HA1, const float* HA2, float* dH2, float* dH1, float* dX,
                          int64_t lddx, const float* mask, int64_t ldm, hipStream_t st,
                          const int* skip, const PolRowArgs* pg = nullptr);
int head_bwd_blocks(int64_t rows);
int launch_ddpg_stats(const float*, int64_t, int, const float*, int64_t, const float*,
                      const float*, int64_t, int64_t, float*, hipStream_t);
int launch_ddpg_target(const float*, const float*, const float*, const float*, int64_t, float,
                       float*, hipStream_t);
void mt_seed_host(uint64_t, uint32_t*);
int mt_randint_host(uint32_t*, int64_t, int64_t, int64_t*);
int launch_mt_randint(uint32_t*, int64_t, int64_t, int64_t*, hipStream_t);
int launch_gather_rows(const float*, int64_t, const int64_t*, int64_t, float*, hipStream_t);
int launch_zfilter_accumulate(const float*, const float*, int, float, float*, float*, float*,
                              hipStream_t);

}  // namespace smi

using namespace smi;

#define SMI_STREAM(s) (static_cast<hipStream_t>(s))
#define REQUIRE(cond, msg) \
  do { if (!(cond)) return set_error(SMI_E_ARG, msg); } while (0)

extern "C" {

int smi_version(void) { return 1; }
const char* smi_last_error(void) { return g_err; }

/* Registers the device scratch used by the multi-workgroup reductions
 * (colstats partials, Adam norm partials).  Not part of the reference API. */
int smi_set_workspace(void* dev_ptr, int64_t bytes) {
  REQUIRE(dev_ptr && bytes > 0, "set_workspace: bad args");
  g_default_ctx.ws = dev_ptr;
  g_default_ctx.bytes = bytes;
  return SMI_OK;
}

smi_context* smi_context_create(void* workspace, int64_t bytes) {
  if (!workspace || bytes <= 0) {
    set_error(SMI_E_ARG, "context_create: bad args");
    return nullptr;
  }
  return new smi_context{workspace, bytes, {true}};
}

int smi_context_make_current(smi_context* ctx) {
  REQUIRE(!ctx || ctx->alive.load(std::memory_order_acquire),
          "context_make_current: the context was destroyed");
  t_ctx = ctx;
  return SMI_OK;
}

int smi_context_destroy(smi_context* ctx) {
  REQUIRE(ctx, "context_destroy: null context");
  if (t_ctx == ctx) t_ctx = nullptr;
  // ws / bytes are never written after create (no race with a reader that
  // passed the alive check): a launch another thread is issuing on this
  // context right now still targets its workspace, which is why the caller
  // frees the workspace only once no thread issues launches with it
  // (include/surreal_mi.h)
  ctx->alive.store(false, std::memory_order_release);   // not freed: see above
  return SMI_OK;
}
int64_t smi_workspace_bytes(void) { return (int64_t)128 << 20; }

#ifdef SMI_FAULT_INJECTION
/* test-only build variant (smi_internal.hpp): select a fault; not declared in
 * include/surreal_mi.h and absent from the product library */
int smi_fault_set(int mode) {
  smi::g_fault = mode;
  return SMI_OK;
}
#endif

/* Per-launch HIP-event timing of the MFMA kernels (GEMM forward / input-grad /
 * weight-grad / split-K reduce, LSTM forward / backward): on != 0 starts a
 * fresh record, 0 stops.  Not part of the reference API (measurement only). */
int smi_kernel_timing(int on) {
  if (!g_kt_ev) {
    g_kt_ev = new hipEvent_t[2 * kKtCap];
    for (int i = 0; i < 2 * kKtCap; ++i)
      if (hipEventCreate(&g_kt_ev[i]) != hipSuccess) return set_error(SMI_E_LAUNCH, "hipEventCreate");
  }
  g_kt = on != 0;
  if (on) g_kt_n.store(0);
  return SMI_OK;
}
/* out4 = {launches, total ms, total algorithmic flops, 0} of class cls
 * (SMI_KT_*); synchronises with the recorded events. */
int smi_kernel_timing_report(int cls, double* out4) {
  if (!out4 || cls < 0 || cls >= KT_COUNT) return set_error(SMI_E_ARG, "kernel_timing_report: bad args");
  double n = 0, ms = 0, fl = 0;
  const int nrec = g_kt_n.load() < kKtCap ? g_kt_n.load() : kKtCap;
  for (int i = 0; i < nrec; ++i) {
    if (g_kt_rec[i].cls != cls) continue;
    if (hipEventSynchronize(g_kt_ev[2 * i + 1]) != hipSuccess) return set_error(SMI_E_LAUNCH, "event sync");
    float t = 0.f;
    if (hipEventElapsedTime(&t, g_kt_ev[2 * i], g_kt_ev[2 * i + 1]) != hipSuccess) continue;
    n += 1; ms += t; fl += g_kt_rec[i].flops;
  }
  out4[0] = n; out4[1] = ms; out4[2] = fl; out4[3] = 0;
  return SMI_OK;
}

int64_t smi_mlp_param_count(int in_dim, int h1, int h2, int out_dim, int with_log_var) {
  return mlp_layout(in_dim, h1, h2, out_dim, with_log_var).fcount;
}

int64_t smi_ppo_fused_lds_bytes(int rows, int obs_dim, int h1, int h2, int act_dim,
                                int critic_h1, int critic_h2) {
  return fused_lds_bytes(rows, obs_dim, h1, h2, act_dim, critic_h1, critic_h2);
}

int64_t smi_ppo_fused_max_params(void) { return ppo_fused_max_params(); }

int smi_zfilter_apply(const float* x, float* out, int64_t rows, int dim, const float* rs,
                      const float* rsq, const float* cnt, float eps, void* stream) {
  REQUIRE(x && out && rs && rsq && cnt && rows >= 0 && dim > 0, "zfilter_apply: bad args");
  return launch_zfilter_apply(x, out, rows, dim, rs, rsq, cnt, eps, SMI_STREAM(stream));
}

int smi_zfilter_update(const float* x, int64_t rows, int dim, int64_t row_stride, float* rs,
                       float* rsq, float* cnt, void* stream) {
  REQUIRE(x && rs && rsq && cnt && rows >= 0 && dim > 0 && row_stride >= dim,
          "zfilter_update: bad args");
  return launch_colstats(x, rows, dim, row_stride, 1, rs, rsq, cnt, SMI_STREAM(stream));
}

int smi_zfilter_colstats(const float* x, int64_t rows, int dim, int64_t row_stride,
                         float* out_sum, float* out_sumsq, void* stream) {
  REQUIRE(x && out_sum && out_sumsq && rows >= 0 && dim > 0 && row_stride >= dim,
          "zfilter_colstats: bad args");
  return launch_colstats(x, rows, dim, row_stride, 0, out_sum, out_sumsq, nullptr,
                         SMI_STREAM(stream));
}


int smi_zfilter_tmajor(const float* obs, const float* obs_next, int B, int T, int S, int D,
                       int use_zf, const float* rs, const float* rsq, const float* cnt, float eps,
                       float* out, int ldo, int form, void* stream) {
  REQUIRE(obs && out && B >= 0 && T >= 1 && S >= 0 && S <= T + 1 && D >= 1 && ldo >= D &&
              form >= 0 && form <= 5,
          "zfilter_tmajor: bad args");
  REQUIRE(S <= T || obs_next, "zfilter_tmajor: obs_next required when S == T + 1");
  REQUIRE(!use_zf || (rs && rsq && cnt), "zfilter_tmajor: filter buffers required");
  if (B == 0 || S == 0) return SMI_OK;
  return launch_zfilter_tmajor(obs, obs_next ? obs_next : obs, B, T, S, D, use_zf, rs, rsq, cnt,
                               eps, out, ldo, form, SMI_STREAM(stream));
}

int smi_reward_filter(float* rewards, int64_t n, float reward_scale, int mode, float* rs,
                      float* rsq, float* cnt, float eps, void* stream) {
  REQUIRE(rewards && n >= 0 && mode >= 0 && mode <= 3, "reward_filter: bad args");
  REQUIRE(mode == 0 || (rs && rsq && cnt), "reward_filter: filter buffers required");
  return launch_reward_filter(rewards, n, reward_scale, mode, rs, rsq, cnt, eps, nullptr,
                              SMI_STREAM(stream));
}

int smi_reward_filter_partial(float* rewards, int64_t n, float reward_scale, int forward,
                              const float* rs, const float* rsq, const float* cnt, float eps,
                              double* sums3, void* stream) {
  REQUIRE(rewards && n >= 0 && sums3 && rs && rsq && cnt, "reward_filter_partial: bad args");
  return launch_reward_filter(rewards, n, reward_scale, (forward ? 1 : 0) | 4,
                              const_cast<float*>(rs), const_cast<float*>(rsq),
                              const_cast<float*>(cnt), eps, sums3, SMI_STREAM(stream));
}

int smi_reward_filter_commit(const double* sums3, float* rs, float* rsq, float* cnt,
                             void* stream) {
  REQUIRE(sums3 && rs && rsq && cnt, "reward_filter_commit: bad args");
  return launch_reward_filter_commit(sums3, rs, rsq, cnt, SMI_STREAM(stream));
}

int smi_diag_gauss(const float* actions, const float* prob0, const float* prob1, int64_t rows,
                   int act_dim, float* loglik, float* lik, float* kl, float* entropy,
                   void* stream) {
  REQUIRE(prob0 && rows >= 0 && act_dim > 0, "diag_gauss: bad args");
  REQUIRE(!(loglik || lik) || actions, "diag_gauss: actions required for loglik");
  REQUIRE(!kl || prob1, "diag_gauss: prob1 required for kl");
  if (rows == 0) return SMI_OK;
  return launch_diag_gauss(actions, prob0, prob1, rows, act_dim, loglik, lik, kl, entropy,
                           SMI_STREAM(stream));
}

int smi_mlp_forward(const float* params, int in_dim, int h1, int h2, int out_dim, int out_act,
                    int with_log_var, const float* x, int64_t rows, int64_t row_stride,
                    int use_zf, const float* zs, const float* zsq, const float* zc, float zeps,
                    float* out, void* stream) {
  REQUIRE(params && x && out && in_dim > 0 && h1 > 0 && h2 > 0 && out_dim > 0 && rows >= 0,
          "mlp_forward: bad args");
  REQUIRE(row_stride >= in_dim, "mlp_forward: row_stride < in_dim");
  REQUIRE(out_act == ACT_NONE || out_act == ACT_TANH, "mlp_forward: out_act must be 0 or 2");
  REQUIRE(!use_zf || (zs && zsq && zc), "mlp_forward: zfilter buffers required");
  return launch_mlp_forward(params, in_dim, h1, h2, out_dim, out_act, with_log_var, x, rows,
                            row_stride, use_zf, zs, zsq, zc, zeps, out, SMI_STREAM(stream));
}

int smi_head_forward(const float* params, int in_dim, int h1, int h2, int out_dim, int tanh_out,
                     const float* x, int64_t ldx, int64_t rows, float* ha1, float* ha2, float* y,
                     float* wT, void* stream) {
  REQUIRE(params && x && ha1 && ha2 && y && rows >= 0 && ldx >= in_dim, "head_forward: bad args");
  const MlpLayout L = mlp_layout(in_dim, h1, h2, out_dim, 0);
  if (!head_fused_ok(in_dim, ldx, h1, h2, out_dim, x, params + L.fW1, params + L.fW2,
                     params + L.fW3))
    return set_error(SMI_E_NOFIT, "head_forward: shape not supported by the fused head");
  return launch_head_fwd_fused(x, ldx, rows, in_dim, params + L.fW1, params + L.fb1, h1,
                               params + L.fW2, params + L.fb2, h2, params + L.fW3,
                               params + L.fb3, out_dim, tanh_out, ha1, ha2, y, out_dim, wT,
                               wT ? wT + (int64_t)in_dim * h1 : nullptr, SMI_STREAM(stream),
                               nullptr);
}

int smi_head_backward_input(const float* params, int in_dim, int h1, int h2, int out_dim,
                            const float* wT, const float* dz, int64_t rows, const float* ha1,
                            const float* ha2, float* dh2, float* dh1, int dx0, int dxn, float* dx,
                            int64_t lddx, const float* mask, int64_t ldm, void* stream) {
  REQUIRE(params && wT && dz && ha1 && ha2 && dh2 && dh1 && rows >= 0 && dx0 >= 0 && dxn >= 0 &&
          dx0 + dxn <= in_dim && (dxn == 0 || (dx && lddx >= dxn)),
          "head_backward_input: bad args");
  const MlpLayout L = mlp_layout(in_dim, h1, h2, out_dim, 0);
  if (dxn > 320 || !head_fused_ok(in_dim, in_dim, h1, h2, out_dim, params, params + L.fW1,
                                  params + L.fW2, params + L.fW3))
    return set_error(SMI_E_NOFIT, "head_backward_input: shape not supported by the fused head");
  return launch_head_bwd_fused(dz, out_dim, rows, params + L.fW3, wT + (int64_t)in_dim * h1, wT,
                               h1, h2, dx0, dxn, ha1, ha2, dh2, dh1, dx, lddx, mask, ldm,
                               SMI_STREAM(stream), nullptr);
}

int smi_ppo_critic_gae(const float* critic_params, int obs_dim, int h1, int h2, int use_zf,
                       const float* zs, const float* zsq, const float* zc, float zeps,
                       const float* obs, const float* obs_next, const float* rewards,
                       const float* dones, int B, int T, const float* gtab, const float* ltab,
                       float gamma, float gamma_T, float* values, float* adv_raw, float* ret,
                       void* stream) {
  REQUIRE(critic_params && obs && obs_next && rewards && dones && gtab && ltab && adv_raw && ret,
          "ppo_critic_gae: null pointer");
  REQUIRE(B >= 1 && T >= 1 && obs_dim >= 1 && h1 >= 1 && h2 >= 1, "ppo_critic_gae: bad dims");
  REQUIRE(!use_zf || (zs && zsq && zc), "ppo_critic_gae: zfilter buffers required");
  return launch_critic_gae(critic_params, obs_dim, h1, h2, use_zf, zs, zsq, zc, zeps, obs,
                           obs_next, rewards, dones, B, T, gtab, ltab, gamma, gamma_T, values,
                           adv_raw, ret, SMI_STREAM(stream));
}

int smi_gae_windows(const float* values, float* values_masked, const float* rewards,
                    const float* dones, int64_t B, int T,
                    int horizon, const float* gtab, const float* ltab, float gamma,
                    float gamma_H, float* adv, float* ret, double* partials, int* n_partials,
                    void* stream) {
  REQUIRE(values && rewards && dones && gtab && ltab && adv && ret, "gae_windows: null pointer");
  REQUIRE(B >= 0 && T >= 1, "gae_windows: bad dims");
  if (B == 0) { if (n_partials) *n_partials = 0; return SMI_OK; }
  return launch_gae_windows(values, values_masked, rewards, dones, B, T, horizon, gtab, ltab, gamma, gamma_H,
                            adv, ret, partials, n_partials, SMI_STREAM(stream));
}

int smi_gae_windows_max_partials(int64_t B, int T) { return gae_windows_max_partials(B, T); }

int smi_moments(const float* x, int64_t n, const double* partials, int n_partials, double* out3,
                void* stream) {
  REQUIRE(out3 && (x || (partials && n_partials > 0)), "moments: bad args");
  return launch_moments(x, n, partials, n_partials, out3, SMI_STREAM(stream));
}

static int check_ppo_args(const smi_ppo_args* a);

int smi_ppo_update_fused(const smi_ppo_args* a, void* stream) {
  const int rc = check_ppo_args(a);
  if (rc) return rc;
  return launch_ppo_fused(a, SMI_STREAM(stream));
}

int64_t smi_ppo_xbuf_floats(int obs_dim, int h1, int h2, int act_dim, int critic_h1,
                            int critic_h2, int mode) {
  return ppo_xbuf_floats(obs_dim, h1, h2, act_dim, critic_h1, critic_h2, mode);
}

static int check_ppo_args(const smi_ppo_args* a) {
  REQUIRE(a, "ppo epochs: null args");
  REQUIRE(a->obs && a->actions && a->behave && a->adv_raw && a->ret && a->actor &&
              a->ref_actor && a->critic && a->actor_m && a->actor_v && a->critic_m &&
              a->critic_v && a->actor_step && a->critic_step && a->hyper && a->stats,
          "ppo epochs: null pointer");
  REQUIRE(!a->use_zf || (a->zf_sum && a->zf_sumsq && a->zf_count && a->rzf_sum &&
                         a->rzf_sumsq && a->rzf_count),
          "ppo epochs: zfilter buffers required");
  REQUIRE(a->mode == 0 || a->mode == 1, "ppo epochs: mode must be 0 (clip) or 1 (adapt)");
  REQUIRE(a->epoch_policy >= 0 && a->epoch_baseline >= 0, "ppo epochs: bad epochs");
  return SMI_OK;
}

int smi_ppo_epoch_grad(const smi_ppo_args* a, int epoch, void* stream) {
  const int rc = check_ppo_args(a);
  if (rc) return rc;
  REQUIRE(epoch >= 0, "ppo_epoch_grad: epoch < 0");
  return launch_ppo_epoch_grad(a, epoch, SMI_STREAM(stream));
}

int smi_ppo_epoch_apply(const smi_ppo_args* a, int epoch, void* stream) {
  const int rc = check_ppo_args(a);
  if (rc) return rc;
  REQUIRE(epoch >= 0, "ppo_epoch_apply: epoch < 0");
  return launch_ppo_epoch_apply(a, epoch, SMI_STREAM(stream));
}

int smi_zfilter_accumulate(const float* sum_in, const float* sumsq_in, int dim, float rows,
                           float* rs, float* rsq, float* cnt, void* stream) {
  REQUIRE(sum_in && sumsq_in && rs && rsq && cnt && dim > 0, "zfilter_accumulate: bad args");
  return launch_zfilter_accumulate(sum_in, sumsq_in, dim, rows, rs, rsq, cnt, SMI_STREAM(stream));
}

int smi_adam_clip(float* params, const float* grad, float* m, float* v, int64_t n, int* step,
                  const float* lr_ptr, float beta1, float beta2, float eps, float weight_decay,
                  float max_norm, float clip_value, const int* skip_flag, float* norm_out,
                  void* stream) {
  REQUIRE(params && grad && m && v && step && lr_ptr && n > 0, "adam_clip: bad args");
  return launch_adam_clip(params, grad, m, v, n, step, lr_ptr, beta1, beta2, eps, weight_decay,
                          max_norm, clip_value, skip_flag, norm_out, SMI_STREAM(stream));
}

int smi_linear_forward(const float* x, int64_t ldx, int rows, int in_dim, const float* w,
                       int64_t ldw, const float* b, int out_dim, int act, float* y, int64_t ldy,
                       void* stream) {
  REQUIRE(x && w && y && rows >= 0 && in_dim > 0 && out_dim > 0, "linear_forward: bad args");
  REQUIRE(ldx >= in_dim && ldy >= out_dim && ldw >= in_dim, "linear_forward: leading dims too small");
  REQUIRE(act == ACT_NONE || act == ACT_RELU || act == ACT_TANH, "linear_forward: act 0/1/2");
  return launch_linear_fwd(x, ldx, rows, in_dim, w, ldw, b, out_dim, act, y, ldy,
                           SMI_STREAM(stream));
}

int smi_linear_forward_cat(const float* x, int64_t ldx, int rows, int in_dim, const float* w,
                           int64_t ldw, const float* b, int out_dim, int act, float* y,
                           int64_t ldy, const float* s, int64_t lds, int s_cols, void* stream) {
  REQUIRE(x && w && y && s && rows >= 0 && in_dim > 0 && out_dim > 0 && s_cols > 0 && lds >= s_cols,
          "linear_forward_cat: bad args");
  REQUIRE(ldx >= in_dim && ldy >= out_dim + s_cols && ldw >= in_dim,
          "linear_forward_cat: leading dims too small");
  REQUIRE(act == ACT_NONE || act == ACT_RELU || act == ACT_TANH, "linear_forward_cat: act 0/1/2");
  return launch_linear_fwd_cat(x, ldx, rows, in_dim, w, ldw, b, out_dim, act, y, ldy, s, lds, s_cols,
                               SMI_STREAM(stream));
}

int smi_linear_backward_input(const float* dy, int64_t ldg, int rows, int out_dim, const float* w,
                              int64_t ldw, int in_dim, const float* relu_mask, int64_t ldm,
                              float* dx, int64_t lddx, void* stream) {
  REQUIRE(dy && w && dx && rows >= 0 && in_dim > 0 && out_dim > 0 && ldw >= in_dim,
          "linear_backward_input: bad args");
  return launch_linear_bwd_dx(dy, ldg, rows, out_dim, w, ldw, in_dim, relu_mask, ldm, dx, lddx,
                              SMI_STREAM(stream));
}

int smi_dw_group_begin(void) { return dw_group_begin(); }

int smi_dw_group_flush(void* stream) { return dw_group_flush(SMI_STREAM(stream)); }

int smi_linear_backward_weight(const float* dy, int64_t ldg, int rows, int out_dim, const float* x,
                               int64_t ldx, int in_dim, float* dw, int64_t lddw, float* db,
                               int accumulate, void* stream) {
  REQUIRE(dy && x && dw && rows >= 0 && in_dim > 0 && out_dim > 0 && lddw >= in_dim,
          "linear_backward_weight: bad args");
  return launch_linear_bwd_dw(dy, ldg, rows, out_dim, x, ldx, in_dim, dw, lddw, db, accumulate,
                              SMI_STREAM(stream));
}

int smi_mse_grad(const float* q, int64_t q_stride, const float* y, int64_t n, float* dq,
                 float* loss, void* stream) {
  REQUIRE(q && y && dq && n > 0, "mse_grad: bad args");
  return launch_mse_grad(q, q_stride, y, n, dq, loss, SMI_STREAM(stream));
}

int smi_neg_mean_grad(const float* q, int64_t q_stride, int64_t n, float* dq, float* loss,
                      void* stream) {
  REQUIRE(q && dq && n > 0, "neg_mean_grad: bad args");
  return launch_neg_mean_grad(q, q_stride, n, dq, loss, SMI_STREAM(stream));
}

int smi_tanh_backward(const float* dy, int64_t ldg, const float* y, int64_t ldy, int64_t rows,
                      int cols, float* dz, int64_t ldz, void* stream) {
  REQUIRE(dy && y && dz && rows >= 0 && cols > 0, "tanh_backward: bad args");
  if (rows == 0) return SMI_OK;
  return launch_tanh_backward(dy, ldg, y, ldy, rows, cols, dz, ldz, SMI_STREAM(stream));
}

int smi_layernorm_forward(const float* x, int64_t ldx, int64_t rows, int n, const float* gamma,
                          const float* beta, float eps, float* y, int64_t ldy, float* mean,
                          float* rstd, void* stream) {
  REQUIRE(x && gamma && beta && y && mean && rstd && rows >= 0, "layernorm_forward: bad args");
  return launch_layernorm_fwd(x, ldx, rows, n, gamma, beta, eps, y, ldy, mean, rstd,
                              SMI_STREAM(stream));
}

int smi_layernorm_backward(const float* dy, int64_t ldg, const float* x, int64_t ldx,
                           const float* mean, const float* rstd, const float* gamma, int64_t rows,
                           int n, int relu_input, float* dx, int64_t lddx, float* dgamma,
                           float* dbeta, void* stream) {
  REQUIRE(dy && x && mean && rstd && gamma && dx && dgamma && dbeta && rows >= 0,
          "layernorm_backward: bad args");
  return launch_layernorm_bwd(dy, ldg, x, ldx, mean, rstd, gamma, rows, n, relu_input, dx, lddx,
                              dgamma, dbeta, SMI_STREAM(stream));
}

int smi_copy_cols(const float* src, int64_t lds, int64_t rows, int cols, float* dst, int64_t ldd,
                  void* stream) {
  REQUIRE(src && dst && rows >= 0 && cols > 0, "copy_cols: bad args");
  if (rows == 0) return SMI_OK;
  return launch_copy_cols(src, lds, rows, cols, dst, ldd, SMI_STREAM(stream));
}

int smi_mlp3_forward_stacked(const float* params, int64_t pstride, const int64_t* offsets6,
                             int in_dim, int h1, int h2, int out_dim, int out_act, const float* x,
                             int64_t ldx, int n, float* y, int64_t ldy, void* stream) {
  REQUIRE(params && offsets6 && x && y && n >= 0 && pstride >= 0 && ldx >= in_dim && ldy >= out_dim &&
              (out_act == 0 || out_act == 1 || out_act == 2),
          "mlp3_forward_stacked: bad args");
  for (int i = 0; i < 6; ++i) REQUIRE(offsets6[i] >= 0, "mlp3_forward_stacked: negative offset");
  if (n == 0) return SMI_OK;
  return launch_mlp3_stacked(params, pstride, offsets6, in_dim, h1, h2, out_dim, out_act, x, ldx, n, y,
                             ldy, SMI_STREAM(stream));
}

int smi_copy_to_host(void* host_dst, const void* src, int64_t nbytes, void* stream) {
  REQUIRE(host_dst && src && nbytes >= 0 && nbytes % 16 == 0 &&
          (reinterpret_cast<uintptr_t>(host_dst) & 15) == 0 &&
          (reinterpret_cast<uintptr_t>(src) & 15) == 0,
          "copy_to_host: 16-byte aligned pointers and a multiple of 16 bytes required");
  if (nbytes == 0) return SMI_OK;
  void* dev = nullptr;
  if (hipHostGetDevicePointer(&dev, host_dst, 0) != hipSuccess || !dev)
    return set_error(SMI_E_ARG, "copy_to_host: destination is not pinned (mapped) host memory");
  return launch_copy_bytes16(src, dev, nbytes / 16, SMI_STREAM(stream));
}

int smi_copy_gather(void* dst, const void* const* srcs, const int64_t* dst_offsets,
                    const int64_t* nbytes, int n, void* stream) {
  REQUIRE(dst && n >= 0 && (n == 0 || (srcs && dst_offsets && nbytes)), "copy_gather: bad args");
  for (int i = 0; i < n; ++i)
    REQUIRE(srcs[i] && nbytes[i] >= 0 && nbytes[i] % 4 == 0 && dst_offsets[i] % 16 == 0 &&
                (reinterpret_cast<uintptr_t>(srcs[i]) & 15) == 0,
            "copy_gather: 16-byte aligned segments of a multiple of 4 bytes required");
  REQUIRE((reinterpret_cast<uintptr_t>(dst) & 15) == 0, "copy_gather: 16-byte aligned destination");
  if (n == 0) return SMI_OK;
  return launch_copy_gather(dst, srcs, dst_offsets, nbytes, n, SMI_STREAM(stream));
}

int smi_soft_update(float* target, const float* src, int64_t n, float tau, void* stream) {
  REQUIRE(target && src && n >= 0, "soft_update: bad args");
  if (n == 0) return SMI_OK;
  return launch_soft_update(target, src, n, tau, SMI_STREAM(stream));
}

int smi_ddpg_stats(const float* actions, int64_t lda, int act_dim, const float* rewards,
                   int64_t rs, const float* y, const float* q, int64_t qs, int64_t n,
                   float* stats4, void* stream) {
  REQUIRE(actions && rewards && y && q && stats4 && n > 0 && act_dim > 0, "ddpg_stats: bad args");
  return launch_ddpg_stats(actions, lda, act_dim, rewards, rs, y, q, qs, n, stats4,
                           SMI_STREAM(stream));
}

int smi_ddpg_target(const float* rewards, const float* dones, const float* q_next,
                    const float* q_next2, int64_t n, float gamma_n, float* y, void* stream) {
  REQUIRE(rewards && dones && q_next && y && n >= 0, "ddpg_target: bad args");
  if (n == 0) return SMI_OK;
  return launch_ddpg_target(rewards, dones, q_next, q_next2, n, gamma_n, y, SMI_STREAM(stream));
}

int smi_mt_seed(uint64_t seed, uint32_t* host_state625) {
  REQUIRE(host_state625, "mt_seed: null state");
  mt_seed_host(seed, host_state625);
  return SMI_OK;
}

int smi_mt_randint_host(uint32_t* host_state625, int64_t n, int64_t batch, int64_t* out) {
  REQUIRE(host_state625 && out && n >= 1 && n <= 0xffffffffLL && batch >= 0,
          "mt_randint_host: bad args");
  return mt_randint_host(host_state625, n, batch, out);
}

int smi_mt_randint(uint32_t* dev_state625, int64_t n, int64_t batch, int64_t* out_indices,
                   void* stream) {
  REQUIRE(dev_state625 && out_indices && batch >= 0, "mt_randint: bad args");
  return launch_mt_randint(dev_state625, n, batch, out_indices, SMI_STREAM(stream));
}

int smi_gather_rows(const float* table, int64_t cols, const int64_t* idx, int64_t batch,
                    float* out, void* stream) {
  REQUIRE(table && idx && out && cols > 0 && batch >= 0, "gather_rows: bad args");
  return launch_gather_rows(table, cols, idx, batch, out, SMI_STREAM(stream));
}


/* ------------------------------------------------ PPO: LSTM policy path */
int64_t smi_lstm_param_count(int in_dim, int hidden) {
  return (int64_t)4 * hidden * in_dim + (int64_t)4 * hidden * hidden + 8 * (int64_t)hidden;
}

int64_t smi_ppo_rnn_scratch_bytes(int B, int T, int horizon, int obs_dim, int rnn_hidden, int h1,
                                  int h2, int act_dim, int critic_h1, int critic_h2, int pix_c,
                                  int pix_h, int pix_w, int cnn_feat, int rnn_layer) {
  return ppo_rnn_scratch_bytes(B, T, horizon, obs_dim, rnn_hidden, rnn_layer, h1, h2, act_dim,
                               critic_h1, critic_h2, pix_c, pix_h, pix_w, cnn_feat);
}

int64_t smi_cnn_param_count(int C, int H, int W, int F) { return cnn_geom(C, H, W, F).total; }

int64_t smi_ppo_rnn_xbuf_floats(int obs_dim, int rnn_hidden, int h1, int h2, int act_dim,
                                int critic_h1, int critic_h2, int pix_c, int pix_h, int pix_w,
                                int cnn_feat, int rnn_layer) {
  const int F = cnn_feat > 0 ? cnn_feat : 0;
  const int hin = rnn_hidden > 0 ? rnn_hidden : obs_dim + F;     // 0: MLP policy on the stem
  const int nl = rnn_layer > 1 ? rnn_layer : 1;
  const int64_t ns = (rnn_hidden > 0 ? smi_lstm_param_count(obs_dim + F, rnn_hidden) +
                                           (nl - 1) * smi_lstm_param_count(rnn_hidden, rnn_hidden)
                                     : 0) +
                     (F > 0 ? smi_cnn_param_count(pix_c, pix_h, pix_w, F) : 0);
  return mlp_layout(hin, h1, h2, act_dim, 1).fcount +
         mlp_layout(hin, critic_h1, critic_h2, 1, 0).fcount + 2 * ns;
}

int64_t smi_cnn_scratch_bytes(int64_t rows, int C, int H, int W, int F) {
  const CnnGeom g = cnn_geom(C, H, W, F);
  return 4 * (rows * g.flat + (int64_t)cnn_bwd_grid(rows) * g.nconv);
}

int smi_cnn_forward(const float* params, const uint8_t* pix, const uint8_t* pix_next, int64_t B,
                    int64_t T, int64_t rows, int C, int H, int W, int F, float* a1, float* a2,
                    float* feat, int64_t ldf, void* stream) {
  REQUIRE(params && pix && a2 && feat && B >= 1 && T >= 1 && rows >= 0 && ldf >= F,
          "cnn_forward: bad args");
  REQUIRE(rows <= B * T || pix_next, "cnn_forward: rows beyond B*T need pix_next");
  const PixRows pr{pix, pix_next, B, T, (int64_t)C * H * W};
  return cnn_forward(params, pr, C, H, W, F, rows, a1, a2, feat, ldf, SMI_STREAM(stream), nullptr);
}

int smi_cnn_backward(const float* params, const uint8_t* pix, const uint8_t* pix_next, int64_t B,
                     int64_t T, int64_t rows, int C, int H, int W, int F, const float* a1,
                     const float* a2, const float* dz, int64_t lddz, float* grad, void* scratch,
                     int64_t scratch_bytes, void* stream) {
  REQUIRE(params && pix && a1 && a2 && dz && grad && scratch && B >= 1 && T >= 1 && rows >= 0 &&
          lddz >= F, "cnn_backward: bad args");
  REQUIRE(rows <= B * T || pix_next, "cnn_backward: rows beyond B*T need pix_next");
  REQUIRE(scratch_bytes >= smi_cnn_scratch_bytes(rows, C, H, W, F), "cnn_backward: scratch too small");
  const CnnGeom g = cnn_geom(C, H, W, F);
  float* dA2 = static_cast<float*>(scratch);
  float* part = dA2 + rows * g.flat;
  const PixRows pr{pix, pix_next, B, T, g.img};
  return cnn_backward(params, pr, C, H, W, F, rows, a1, a2, dz, lddz, grad, dA2, part,
                      SMI_STREAM(stream), nullptr);
}

int smi_ppo_rnn_phase(const smi_ppo_rnn_args* a, int phase, int epoch, void* stream) {
  REQUIRE(a, "ppo_rnn: null args");
  REQUIRE(a->rnn_layer >= 0 && a->rnn_layer <= 3 && (a->rnn_layer <= 1 || a->rnn_hidden > 0),
          "ppo_rnn: rnn_layer must be in [1, 3] (0 = 1)");
  REQUIRE(a->B >= 1 && a->T >= 1 && a->horizon >= 1 && a->horizon <= a->T, "ppo_rnn: bad B/T/horizon");
  REQUIRE(a->obs_dim >= (a->cnn_feat > 0 ? 0 : 1) && a->obs_dim <= 128,
          "ppo_rnn: obs_dim must be in [1, 128] ([0, 128] with a pixel stem)");
  REQUIRE(a->cnn_feat <= 0 || (a->pixels && a->pixels_next),
          "ppo_rnn: pixel stem needs pixels and pixels_next");
  REQUIRE(!(a->use_zf && a->obs_dim == 0), "ppo_rnn: z-filter needs low-dim observations");
  REQUIRE(a->rnn_hidden >= 0 && a->rnn_hidden <= 256,
          "ppo_rnn: rnn_hidden must be in [0, 256] (0: MLP policy over the stem input)");
  REQUIRE(a->rnn_hidden > 0 || a->horizon == a->T,
          "ppo_rnn: the MLP policy (rnn_hidden 0) uses horizon == n_step (one window)");
  REQUIRE(a->act_dim >= 1 && a->act_dim <= 32, "ppo_rnn: act_dim must be in [1, 32]");
  REQUIRE(a->h1 >= 1 && a->h2 >= 1 && a->critic_h1 >= 1 && a->critic_h2 >= 1, "ppo_rnn: bad hidden sizes");
  REQUIRE((a->obs_dim == 0 || (a->obs && a->obs_next)) && a->actions && a->rewards && a->dones &&
          a->behave && (a->rnn_hidden == 0 || (a->h0 && a->c0)), "ppo_rnn: null batch pointer");
  REQUIRE(a->actor && a->critic && a->ref_actor &&
          ((a->rnn_hidden == 0 && a->cnn_feat <= 0) || (a->lstm && a->ref_lstm)),
          "ppo_rnn: null params");
  REQUIRE(a->actor_m && a->actor_v && a->critic_m && a->critic_v && a->actor_step &&
          a->critic_step && a->hyper && a->gamma_tab && a->lam_tab, "ppo_rnn: null optimizer state");
  REQUIRE(a->stats && a->kl_record && a->kl_count && a->moments && a->pstat && a->xbuf && a->zbuf &&
          a->scratch, "ppo_rnn: null output/exchange buffer");
  REQUIRE(!a->use_zf || (a->zf_sum && a->zf_sumsq && a->zf_count && a->rzf_sum && a->rzf_sumsq &&
                         a->rzf_count), "ppo_rnn: zfilter buffers required");
  REQUIRE(a->B_global >= a->B, "ppo_rnn: B_global < B");
  return ppo_rnn_phase(*a, phase, epoch, SMI_STREAM(stream));
}

int smi_lstm_forward(const float* xproj, const float* w_hh, const float* b_hh, const float* h0,
                     const float* c0, int S, int B, int H, float* hbuf, float* cbuf,
                     float* gates_act, void* stream) {
  REQUIRE(xproj && w_hh && b_hh && h0 && c0 && hbuf && S >= 0 && B >= 0 && H >= 1,
          "lstm_forward: bad args");
  return launch_lstm_fwd(xproj, w_hh, b_hh, h0, c0, S, B, H, hbuf, cbuf, gates_act,
                         SMI_STREAM(stream), nullptr);
}

int smi_lstm_forward_x(const float* x, int64_t ldx, int din, const float* w_ih,
                       const float* b_ih, const float* w_hh, const float* b_hh, const float* h0,
                       const float* c0, int S, int B, int H, float* hbuf, float* cbuf,
                       float* gates_act, float* xproj_scratch, void* stream) {
  REQUIRE(x && w_ih && b_ih && w_hh && b_hh && h0 && c0 && hbuf && S >= 0 && B >= 0 && H >= 1 &&
          din >= 1 && ldx >= din, "lstm_forward_x: bad args");
  const hipStream_t st = SMI_STREAM(stream);
  const int rf = launch_lstm_fwd_x(x, ldx, din, w_ih, b_ih, w_hh, b_hh, h0, c0, S, B, H, hbuf, cbuf,
                                   gates_act, st, nullptr, 0);
  if (rf != SMI_E_NOFIT) return rf;
  REQUIRE(xproj_scratch, "lstm_forward_x: the unfused form needs xproj_scratch [S][B][4H]");
  const int rc = launch_linear_fwd(x, ldx, S * B, din, w_ih, din, b_ih, 4 * H, ACT_NONE,
                                   xproj_scratch, 4 * H, st, nullptr);
  if (rc) return rc;
  return launch_lstm_fwd(xproj_scratch, w_hh, b_hh, h0, c0, S, B, H, hbuf, cbuf, gates_act, st,
                         nullptr);
}

int smi_lstm_backward(const float* dh, const float* gates_act, const float* cbuf,
                      const float* w_hh, int S, int B, int H, float* dgates, void* stream) {
  REQUIRE(dh && gates_act && cbuf && w_hh && dgates && S >= 0 && B >= 0 && H >= 1,
          "lstm_backward: bad args");
  return launch_lstm_bwd(dh, gates_act, cbuf, w_hh, S, B, H, dgates, SMI_STREAM(stream), nullptr);
}

}  // extern "C"
