/*
 * surreal_mi.h — C ABI of the MI355X-native SURREAL centralized-learner hot path.
 *
 * One shared library (libsurreal_mi.so, gfx950 code objects) exposes plain
 * `extern "C"` entry points.  Every entry point:
 *   - takes caller-owned DEVICE pointers (HBM) plus explicit sizes/strides;
 *   - takes the hipStream_t to enqueue on as `void* stream` (NULL = default);
 *   - never allocates, never synchronises (safe inside hipGraph capture);
 *   - returns 0 on success, a negative SMI_E* code on argument errors, or
 *     -(hipError_t) if the launch failed; smi_last_error() holds a message.
 *
 * Each function names the reference interface it replaces (file:line in
 * tanwanirahul/surreal).  Host-side mirrors of the reference Python classes
 * live in surreal_amd/ (learner.py, model.py, replay.py) and call these.
 *
 * Parameter-buffer layout ("flat MLP layout", used by every MLP argument):
 *   W1[H1][IN] b1[H1] W2[H2][H1] b2[H2] W3[OUT][H2] b3[OUT] (+ log_var[OUT] for
 *   PPO actors).  Row-major, fp32, i.e. torch nn.Linear (out, in) weights laid
 *   end to end — see smi_mlp_param_count().
 */
#ifndef SURREAL_MI_H
#define SURREAL_MI_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------------------------------------------------------- errors */
#define SMI_OK            0
#define SMI_E_ARG        -1   /* bad size / null pointer / unsupported dims */
#define SMI_E_NOFIT      -2   /* problem does not fit the requested kernel variant */
#define SMI_E_LAUNCH     -3   /* hip launch error (see smi_last_error) */

int         smi_version(void);
const char* smi_last_error(void);

/* Device scratch for the multi-workgroup reductions (ZFilter column partials,
 * Adam norm partials, split-K GEMM partials).  The caller allocates
 * smi_workspace_bytes() of device memory and registers it.
 *
 * Re-entrancy (SURVEY §8(b) Threading: the reference issues DDPG preprocess
 * GPU work from the prefetch thread while learn() runs, data_fetcher.py:47-58).
 * Kernels themselves are stateless; the only host state a launch consults is
 * (a) the workspace its partials go to and (b) the queue of a grouped weight-
 * gradient launch.  (b) is thread-local (smi_dw_group_begin/flush bracket a
 * call sequence on one thread).  (a) belongs to an smi_context: each object
 * that launches work (a learner, an agent batch) owns one context with its
 * own workspace and makes it current on the calling thread before its calls;
 * launches then use the calling thread's current context, so two objects on
 * two streams (or two threads) never share partial buffers.  With no current
 * context a thread uses the default workspace of smi_set_workspace. */
int64_t smi_workspace_bytes(void);
int     smi_set_workspace(void* dev_ptr, int64_t bytes);
typedef struct smi_context smi_context;
smi_context* smi_context_create(void* workspace, int64_t bytes);   /* NULL on bad args */
int          smi_context_make_current(smi_context* ctx);            /* this thread; NULL = default */
/* Marks ctx dead (its 24-byte handle is kept, never freed): a thread that
 * still has it current falls back to the default workspace for its LATER
 * launches; making a dead context current is an error.  A launch that another
 * thread is issuing on ctx concurrently with the destroy may still use its
 * workspace: free the workspace only after every thread that had ctx current
 * has finished issuing launches with it (the Python owner, _lib.Context, is
 * referenced from each thread's current-context slot, so the workspace lives
 * while any thread has the context current). */
int          smi_context_destroy(smi_context* ctx);

/* Measurement only (not part of the reference API): per-launch HIP-event
 * timing of the MFMA kernels and of the HBM-bound streaming kernels of the
 * RNN learner phases, by class.  smi_kernel_timing(1) starts a fresh record,
 * (0) stops; smi_kernel_timing_report(cls, out4) -> {launches, total ms, total
 * algorithmic work, 0}: flops for classes 0-7, bytes for classes 8-13. */
#define SMI_KT_GEMM_FWD    0
#define SMI_KT_GEMM_DX     1
#define SMI_KT_GEMM_DW     2
#define SMI_KT_GEMM_REDUCE 3
#define SMI_KT_LSTM_FWD    4
#define SMI_KT_LSTM_BWD    5
#define SMI_KT_CNN_FWD     6
#define SMI_KT_CNN_BWD     7
#define SMI_KT_GAE         8    /* windowed GAE (bytes)                         */
#define SMI_KT_POLICY_STATS 9   /* policy loss / KL statistics rows (bytes)     */
#define SMI_KT_POLICY_GRAD 10   /* policy loss gradient rows (bytes)            */
#define SMI_KT_VALUE_ROWS  11   /* value loss rows (bytes)                      */
#define SMI_KT_ADAM        12   /* grad-norm partials + Adam (bytes)            */
#define SMI_KT_ZF_TMAJOR   13   /* ZFilter apply into the time-major stem input */
int smi_kernel_timing(int on);
int smi_kernel_timing_report(int cls, double* out4);

/* Measurement only: what the box delivers, beside bench.py's timed region
 * (calib_kernels.hip).  smi_calib_mfma: n_wg workgroups of 4 waves, each
 * wave `iters` x 4 v_mfma_f32_32x32x2_f32 on random register operands
 * (16384 flops per wave and iteration); out[n_wg * 256] keeps the sums live,
 * stamps[2 n_wg] = per workgroup (d s_memtime, d s_memrealtime), i.e. the
 * in-kernel clock d_memtime / d_realtime x 100 MHz.  smi_calib_stream:
 * y[i] = x[i] * (1 + 1e-7), n floats (8 bytes moved per float), float4
 * nontemporal.  smi_clock_probe: one wave sleeping in a loop until *flag != 0
 * (smi_clock_probe_stop, on another stream) or max_ticks of the 100 MHz
 * counter pass; out3 = {d s_memtime, d s_memrealtime, timed_out}. */
int smi_calib_mfma(int n_wg, int iters, float* out, long long* stamps, void* stream);
int smi_calib_stream(const float* x, float* y, int64_t n, void* stream);
int smi_clock_probe(const int* flag, long long max_ticks, long long* out3, void* stream);
int smi_clock_probe_stop(int* flag, int value, void* stream);

/* --------------------------------------------------------------- layouts */
/* Number of floats in a flat MLP buffer (in -> h1 -> h2 -> out [+ log_var]). */
int64_t smi_mlp_param_count(int in_dim, int h1, int h2, int out_dim, int with_log_var);

/* Dynamic LDS bytes the fused small-batch PPO kernel needs; more than 163840
 * (160 KiB, one CU) means it does not fit and the modular path must be used. */
int64_t smi_ppo_fused_lds_bytes(int rows, int obs_dim, int h1, int h2, int act_dim,
                                int critic_h1, int critic_h2);

/* Largest per-network parameter count smi_ppo_update_fused accepts (its Adam
 * moments are register-resident); larger networks use the epoch phases
 * (smi_ppo_epoch_grad / smi_ppo_epoch_apply) even on a single GPU. */
int64_t smi_ppo_fused_max_params(void);

/* ----------------------------------------------------------- ZFilter ops */
/* Replaces ZFilter.forward (surreal/model/z_filter.py:59-79):
 *   out = clamp((x - sum/count) / max(sqrt(sumsq/count - mean^2), eps), -5, 5)
 * x, out: [rows][dim] (may alias). */
int smi_zfilter_apply(const float* x, float* out, int64_t rows, int dim,
                      const float* running_sum, const float* running_sumsq,
                      const float* count, float eps, void* stream);

/* Replaces ZFilter.z_update (surreal/model/z_filter.py:44-57):
 *   running_sum += sum_r x[r], running_sumsq += sum_r x[r]^2, count += rows.
 * Rows are read with an explicit row stride (floats) so obs[:,0,:] can be passed
 * without a copy. */
int smi_zfilter_update(const float* x, int64_t rows, int dim, int64_t row_stride,
                       float* running_sum, float* running_sumsq, float* count,
                       void* stream);

/* Column sums / sums of squares only (no buffer update): out_sum[dim],
 * out_sumsq[dim] — used by the data-parallel learner before its all-reduce. */
int smi_zfilter_colstats(const float* x, int64_t rows, int dim, int64_t row_stride,
                         float* out_sum, float* out_sumsq, void* stream);

/* The learner's time-major z-filtered input (ZFilter.forward, z_filter.py:59-79,
 * as ppo_net.py:146-149 applies it to obs[:, t] before the LSTM, with the
 * obs_next row appended as ppo.py:385-386 builds the critic's input):
 *   out[t*B + b][c] = zf(obs[b][t][c])  for t < T,  zf(obs_next[b][c]) for t == T,
 * for t < S (S <= T + 1), c < D, rows ldo floats apart; zf = the clamp of
 * smi_zfilter_apply with the (running_sum, running_sumsq, count) stats, or the
 * identity when use_zf == 0.  form: 0 = the learner's choice, 1 = row kernel,
 * 2 = float2 tile transpose, 3 = float4 tile transpose, 4 / 5 = form 3
 * writing whole rows (zeros in columns D..ldo-1; needs ldo == D rounded up to
 * 4), pipelined over a resident grid / one tile per workgroup.  Forms 2 / 3-5
 * need 8- / 16-byte aligned pointers (SMI_E_ARG otherwise); columns < D are
 * bit-identical across forms, and forms 0-3 leave columns D..ldo-1 untouched. */
int smi_zfilter_tmajor(const float* obs, const float* obs_next, int B, int T, int S, int D,
                       int use_zf, const float* running_sum, const float* running_sumsq,
                       const float* count, float eps, float* out, int ldo, int form,
                       void* stream);

/* Replaces RewardFilter.forward / RewardFilter.update
 * (surreal/model/reward_filter.py:18-56) as used by _preprocess_batch_ppo
 * (ppo.py:452-456): rewards *= reward_scale, then by `mode` bits
 *   1 = forward (whiten with the stats from before this call),
 *   2 = update  (count += n; running_sum += sum; running_sumsq = sum of squares —
 *                the reference's `=` instead of `+=` at reward_filter.py:42).
 * mode 0 only scales.  In place on rewards[n]. */
int smi_reward_filter(float* rewards, int64_t n, float reward_scale, int mode,
                      float* running_sum, float* running_sumsq, float* count,
                      float eps, void* stream);

/* RewardFilter under data parallelism (one process per GPU; the reference has
 * one learner, reward_filter.py:33-42 over the whole batch).  _partial scales
 * (and, if forward != 0, whitens with the pre-update stats) like
 * smi_reward_filter, but leaves the filter untouched and writes this rank's
 * {sum(r), sum(r*r), n} (fp64) to sums3[3].  After a SUM all-reduce of sums3
 * over the ranks, _commit applies the reference update with the global sums:
 * count += n, running_sum += sum, running_sumsq = sum of squares. */
int smi_reward_filter_partial(float* rewards, int64_t n, float reward_scale, int forward,
                              const float* running_sum, const float* running_sumsq,
                              const float* count, float eps, double* sums3, void* stream);
int smi_reward_filter_commit(const double* sums3, float* running_sum, float* running_sumsq,
                             float* count, void* stream);

/* ---------------------------------------------------------- DiagGauss ops */
/* Replaces DiagGauss.loglikelihood / likelihood / kl / entropy
 * (surreal/model/ppo_net.py:29-72).  prob rows are [mean(A) | std(A)].
 * Each output is [rows]; pass NULL for outputs you do not need.
 *   loglik[r] = -0.5*sum(((a-mu)/sd)^2) - 0.5*log(2pi)*A - sum(log sd)
 *   lik[r]    = max(exp(loglik[r]), 1e-5)
 *   kl[r]     = KL(prob0[r] || prob1[r])
 *   ent[r]    = 0.5*sum(log sd) + 0.5*log(2 pi e)*A            (of prob0) */
int smi_diag_gauss(const float* actions, const float* prob0, const float* prob1,
                   int64_t rows, int act_dim,
                   float* loglik, float* lik, float* kl, float* entropy, void* stream);

/* ------------------------------------------------------------ MLP forward */
/* Replaces PPOModel.forward_actor / forward_critic for the low-dim MLP model
 * (surreal/model/ppo_net.py:253-315, builders.py:86-175):
 *   x -> [ZFilter] -> Linear-ReLU-Linear-ReLU-Linear [-Tanh]
 * act: 0 none (critic), 2 tanh (actor mean).  If with_log_var, out has 2*OUT
 * columns: [tanh(...) | exp(log_var)] exactly like PPO_ActorNetwork.forward.
 * zf_* may be NULL when use_zf == 0.  x rows are strided (row_stride floats). */
int smi_mlp_forward(const float* params, int in_dim, int h1, int h2, int out_dim,
                    int out_act, int with_log_var,
                    const float* x, int64_t rows, int64_t row_stride,
                    int use_zf, const float* zf_sum, const float* zf_sumsq,
                    const float* zf_count, float zf_eps,
                    float* out, void* stream);

/* The learner's head passes over tall activation matrices, each ONE launch
 * (head_kernels.hip; the RNN learner's phases call them internally):
 *   forward:  ha1 = relu(x W1^T + b1), ha2 = relu(ha1 W2^T + b2),
 *             y = act(ha2 W3^T + b3) (tanh_out: tanh) — PPO_ActorNetwork /
 *             PPO_CriticNetwork (builders.py:86-175) without log_var;
 *             wT (nullable, in*h1 + h1*h2 floats) receives W1^T | W2^T for the
 *             backward below.
 *   backward_input: from dz = dL/d(pre-activation of the last layer):
 *             dh2 = (dz W3) * [ha2 > 0], dh1 = (dh2 W2) * [ha1 > 0],
 *             dx[:, 0:dxn] = (dh1 W1[:, dx0:dx0+dxn]) (* [mask > 0] when mask)
 *             using the forward's wT; dxn == 0: no dx.
 * params: the flat [W1 b1 W2 b2 W3 b3] layout of smi_mlp_forward.  Rows of x
 * are ldx floats apart.  Shapes: in, h1, h2 multiples of 4 in [4, 512] (in
 * <= 320), out <= 16, dxn <= 320, 16-byte aligned x / params; otherwise
 * SMI_E_NOFIT (use smi_linear_* per layer). */
int smi_head_forward(const float* params, int in_dim, int h1, int h2, int out_dim, int tanh_out,
                     const float* x, int64_t ldx, int64_t rows, float* ha1, float* ha2,
                     float* y, float* wT, void* stream);
int smi_head_backward_input(const float* params, int in_dim, int h1, int h2, int out_dim,
                            const float* wT, const float* dz, int64_t rows, const float* ha1,
                            const float* ha2, float* dh2, float* dh1, int dx0, int dxn, float* dx,
                            int64_t lddx, const float* mask, int64_t ldm, void* stream);

/* ------------------------------------------------------- PPO: GAE/returns */
/* Replaces PPOLearner._gae_and_return, non-RNN branch
 * (surreal/learner/ppo.py:355-387,408-418): the critic forward over
 * cat(obs, obs_next) (B*(T+1) rows, ZFilter fused into the first layer),
 * done-masking values[:,1:] *= 1-dones, then the windowed sums
 *   ret[b] = sum_t g[t]*r[b,t] + Vm[b,T]*gamma_T
 *   adv[b] = sum_t (td[b,t]*g[t])*l[t],  td = r + gamma*Vm[:,1:] - Vm[:,:-1]
 * g/l are torch.pow(float32) tables (length T) computed by the host exactly as
 * the reference does (ppo.py:372-374); gamma_T = float(gamma**T).
 * Outputs: values[B][T+1] (masked; may be NULL), adv_raw[B] (NOT normalised),
 * ret[B].  obs: [B][T][D] obs_next: [B][1][D] rewards/dones: [B][T]. */
int smi_ppo_critic_gae(const float* critic_params, int obs_dim, int h1, int h2,
                       int use_zf, const float* zf_sum, const float* zf_sumsq,
                       const float* zf_count, float zf_eps,
                       const float* obs, const float* obs_next,
                       const float* rewards, const float* dones, int B, int T,
                       const float* gamma_tab, const float* lam_tab,
                       float gamma, float gamma_T,
                       float* values, float* adv_raw, float* ret, void* stream);

/* Replaces the windowed GAE of the RNN branch (ppo.py:389-406) — and, with
 * horizon == T, the non-RNN sums — given already computed critic values
 * values[B][T+1].  The done mask values[:,1:] *= 1-dones (ppo.py:387) is
 * applied on the fly; values_masked (may be NULL, may alias values) receives
 * the masked values when the caller wants them:
 *   E = T - horizon + 1 windows per segment, s in [0,E):
 *   ret[b,s] = sum_{k<H} g[k]*r[b,s+k] + Vm[b,s+H]*gamma_H
 *   adv[b,s] = sum_{k<H} (td[b,s+k]*g[k])*l[k]
 * HBM-bound streaming kernel: 16-byte coalesced loads staged through LDS.  adv_partials receives per-workgroup
 * (sum, sumsq) doubles; *n_partials is set on return (host-side value). */
int smi_gae_windows(const float* values, float* values_masked,
                    const float* rewards, const float* dones,
                    int64_t B, int T, int horizon,
                    const float* gamma_tab, const float* lam_tab,
                    float gamma, float gamma_H,
                    float* adv, float* ret, double* adv_partials,
                    int* n_partials, void* stream);
int smi_gae_windows_max_partials(int64_t B, int T);

/* (sum, sum of squares, count) in fp64 of x[n] -> out[3]; if partials != NULL
 * and n_partials > 0 the (sum, sumsq) pairs are reduced instead of x (count = n).
 * Deterministic (fixed order).  Feeds the advantage normaliser (ppo.py:413-416). */
int smi_moments(const float* x, int64_t n, const double* partials, int n_partials,
                double* out3, void* stream);

/* ------------------------------------------------- PPO: fused small batch */
/* The whole PPO optimisation of one learn() call for a non-RNN low-dim model
 * when the batch fits one CU (rows <= 256 and params fit LDS):
 * PPOLearner._optimize (surreal/learner/ppo.py:487-586) minus GAE/z_update:
 *   advantage normalisation (ppo.py:413-416), ref_pol (ppo.py:539), up to
 *   epoch_policy actor updates with the KL early stop (ppo.py:541-557; clip
 *   ppo.py:194-248 or adapt ppo.py:250-309, clip_grad_norm_, Adam), and
 *   epoch_baseline critic updates (ppo.py:311-353,561-562), plus the
 *   statistics of ppo.py:568-576.
 * Workgroup 0 runs the policy loop, workgroup 1 the value loop (independent
 * parameter sets in the reference).  Hyper-parameters that the host may change
 * between calls (clip_epsilon, beta, learning rates) are read from `hyper`
 * (device memory), so the call can be captured once in a hipGraph.
 * See struct smi_ppo_args for every field. */
typedef struct smi_ppo_args {
  /* dims */
  int B;              /* policy rows (segments)                         */
  int obs_dim, h1, h2, act_dim;
  int critic_h1, critic_h2;
  int epoch_policy, epoch_baseline;
  int mode;           /* 0 = clip, 1 = adapt                             */
  int norm_adv;
  int clip_actor_grad, clip_critic_grad;
  int use_zf;
  /* inputs: row r of each is base + r*stride (floats) */
  const float* obs;      int64_t obs_stride;      /* obs[:,0,:]          */
  const float* actions;  int64_t act_stride;      /* actions[:,0,:]      */
  const float* behave;   int64_t beh_stride;      /* pds[:,0,:] (2A)     */
  const float* adv_raw;                           /* [B]                 */
  const double* adv_moments;  /* NULL: normalise over these B rows; else
                                 [3] = global (sum, sum of squares, count)
                                 of the raw advantages (data parallel) */
  const float* ret;                               /* [B]                 */
  /* ZFilter buffers of the model and of ref_target_model */
  const float* zf_sum;  const float* zf_sumsq;  const float* zf_count;
  const float* rzf_sum; const float* rzf_sumsq; const float* rzf_count;
  float zf_eps;
  /* parameters (flat MLP layout), Adam state, step counters */
  float* actor;  const float* ref_actor;  float* critic;
  float* actor_m; float* actor_v; float* critic_m; float* critic_v;
  int* actor_step; int* critic_step;
  /* device hyper-parameters: see SMI_HYP_* */
  const float* hyper;
  /* constants */
  double kl_target;           /* python float semantics in comparisons */
  float kl_cutoff_coeff;
  float actor_max_norm, critic_max_norm;
  float actor_wd, critic_wd;
  float beta1, beta2, adam_eps;
  /* outputs */
  float* stats;                /* [SMI_ST_COUNT]                       */
  float* kl_record; int* kl_count; int kl_capacity;
  /* data-parallel epochs (smi_ppo_epoch_grad / smi_ppo_epoch_apply) */
  int64_t B_global;            /* rows over all ranks (0: = B)         */
  float* xbuf;                 /* exchange buffer, smi_ppo_xbuf_floats */
  int* dp_state;               /* [4] zeroed by the caller per learn()  */
  /* optional (NULL: not written): the advantages exactly as the policy epochs
     use them (normalised on device when norm_adv, ppo.py:413-416), [B] */
  float* adv_out;
} smi_ppo_args;

/* device hyper-parameter slots (float) */
#define SMI_HYP_CLIP_EPS   0
#define SMI_HYP_BETA       1
#define SMI_HYP_LR_ACTOR   2
#define SMI_HYP_LR_CRITIC  3
#define SMI_HYPX_CLIP_LO   4   /* float(1 - clip_epsilon) (torch.clamp bound) */
#define SMI_HYPX_CLIP_HI   5   /* float(1 + clip_epsilon)                      */
#define SMI_HYP_COUNT      6

/* statistics slots written by the PPO kernels (float) */
#define SMI_ST_SURR_LOSS        0   /* _surr_loss                          */
#define SMI_ST_CLIP_SURR_LOSS   1   /* _clip_surr_loss (clip mode)         */
#define SMI_ST_KL_LOSS_ADAPT    2   /* _kl_loss_adapt (adapt mode)         */
#define SMI_ST_ENTROPY          3   /* _entropy                            */
#define SMI_ST_POL_KL           4   /* _pol_kl (after the last update)     */
#define SMI_ST_GRAD_NORM_ACTOR  5   /* grad_norm_actor                     */
#define SMI_ST_VAL_LOSS         6   /* _val_loss                           */
#define SMI_ST_VAL_EXPL_VAR     7   /* _val_explained_var                  */
#define SMI_ST_GRAD_NORM_CRITIC 8   /* grad_norm_critic                    */
#define SMI_ST_AVG_RETURN       9   /* _avg_return_targ                    */
#define SMI_ST_AVG_LOG_SIG     10   /* _avg_log_sig                        */
#define SMI_ST_AVG_BEHAVE_LIK  11   /* _avg_behave_likelihood              */
#define SMI_ST_AVG_IS_WEIGHT   12   /* _avg_is_weight                      */
#define SMI_ST_REF_BEHAVE_DIFF 13   /* _ref_behave_diff                    */
#define SMI_ST_EPOCHS_RUN      14   /* policy updates applied (float)      */
#define SMI_ST_POL_KL_ADAPT    15   /* kl used by the adapt loss           */
#define SMI_ST_COUNT           16

int smi_ppo_update_fused(const smi_ppo_args* args, void* stream);

/* Data-parallel form of the same epochs (one process per GPU, the batch
 * sharded on the segment axis).  Phase e in [0, max(E+1, Ev))
 * of one learn() is
 *     smi_ppo_epoch_grad(args, e)  -> this rank's share of the gradients and
 *                                     statistic sums in args->xbuf
 *     all-reduce(SUM) of xbuf (smi_ppo_xbuf_floats floats) across ranks
 *     smi_ppo_epoch_apply(args, e) -> KL early stop / adapt coefficient from
 *                                     the global KL, clip_grad_norm_ + Adam on
 *                                     the summed gradients, statistics
 * Per-row gradient weights use 1/B_global, so the all-reduced sum is the
 * gradient of the reference's mean over the global batch.  args->adv_moments
 * must hold the all-reduced (sum, sumsq, count) of the raw advantages.
 * The early-stop decision is data dependent but identical on every rank, and
 * later phases become no-ops on device: the host issues the same sequence on
 * every rank with no synchronisation. */
int64_t smi_ppo_xbuf_floats(int obs_dim, int h1, int h2, int act_dim, int critic_h1,
                            int critic_h2, int mode);
int smi_ppo_epoch_grad(const smi_ppo_args* args, int epoch, void* stream);
int smi_ppo_epoch_apply(const smi_ppo_args* args, int epoch, void* stream);

/* ------------------------------------------- PPO: LSTM policy (RNN branch) */
/* PPOLearner._optimize with if_rnn_policy (surreal/learner/ppo.py:487-586,
 * 389-406; PPOModel with the nn.LSTM stem, ppo_net.py:137-152,253-315):
 * obs -> ZFilter -> LSTM(h0, c0) -> actor / critic MLP heads, on the MFMA GEMM
 * engine and persistent LSTM sequence kernels (one workgroup per 16 segments,
 * all steps in one launch).  Activations are kept time-major ([step][segment]).
 * One learn() is a fixed sequence of phases (SMI_RNN_PH_*) issued by the host
 * in the same order on every rank; between some phases a data-parallel caller
 * all-reduces (SUM) the buffer named in the phase table (include order):
 *   GAE              -> all-reduce moments (double[3], smi_ppo_rnn_args.moments)
 *   PREP             (reference-policy forward; with prep_independent == 0
 *                    after GAE on the same stream — at one segment per
 *                    workgroup GAE then runs PREP's recurrence in its own
 *                    launch and PREP only the reference head; with
 *                    prep_independent != 0 GAE leaves PREP's work alone and
 *                    the caller may issue PREP on a second stream)
 *   POLICY_FWD(e)    e = 0..epoch_policy: forward + loss sums -> all-reduce pstat
 *   POLICY_DECIDE(e) KL early stop / adapt coefficient / statistics from pstat
 *                    (with B_global == B, one rank, POLICY_FWD already decides
 *                    in the same launch as its reduction and this phase is a no-op)
 *   POLICY_BWD(e)    e < epoch_policy: backward -> all-reduce actor grads
 *                    (xbuf[0 : nA], nA = actor params + lstm params)
 *   POLICY_APPLY(e)  clip_grad_norm_ + Adam over [actor | lstm]
 *   VALUE_GRAD(e)    e = 0..epoch_baseline-1 -> all-reduce critic grads
 *                    (xbuf[nA : nA + nC], nC = critic params + lstm params)
 *   VALUE_APPLY(e)   clip_grad_norm_ + Adam over [critic | lstm]
 *   ZSTATS           column sums of obs_iter -> all-reduce zbuf (value sums of
 *                    the last value epoch + 2D ZFilter sums, doubles)
 *   ZAPPLY           z_update from the (reduced) column sums
 * The KL early stop (ppo.py:556) and the adapt penalty branch (ppo.py:275) are
 * decided on device from the (global) sums; skipped phases are no-ops, so the
 * host never synchronises.  The LSTM parameters belong to both optimizers
 * (ppo_net.py:202-224): actor_m/v and critic_m/v each cover [head | lstm].
 * Flat LSTM layout (nn.LSTM parameter order): W_ih[4H][D] W_hh[4H][H] b_ih[4H]
 * b_hh[4H], gates in torch order (i, f, g, o). */
#define SMI_RNN_PH_GAE           0
#define SMI_RNN_PH_PREP          1
#define SMI_RNN_PH_POLICY_FWD    2
#define SMI_RNN_PH_POLICY_BWD    3
#define SMI_RNN_PH_POLICY_APPLY  4
#define SMI_RNN_PH_VALUE_GRAD    5
#define SMI_RNN_PH_VALUE_APPLY   6
#define SMI_RNN_PH_ZSTATS        7
#define SMI_RNN_PH_ZAPPLY        8
#define SMI_RNN_PH_POLICY_DECIDE 9

typedef struct smi_ppo_rnn_args {
  /* dims (local batch) */
  int B, T, horizon;                 /* segments on this rank, n_step, horizon */
  int obs_dim, rnn_hidden;           /* D, H (rnn_layer LSTM layers).  H == 0: no LSTM — the heads
                                        read the stem input [zfilter(low) | cnn] directly
                                        (the non-RNN pixel model); then horizon == T (one
                                        window: ppo.py:408-418) and only step 0 of each
                                        segment trains (ppo.py:532-535) */
  int h1, h2, act_dim;               /* actor head                            */
  int critic_h1, critic_h2;
  int epoch_policy, epoch_baseline;
  int mode, norm_adv, clip_actor_grad, clip_critic_grad, use_zf;
  int64_t B_global;                  /* segments over all ranks               */
  /* batch as MultistepAggregatorWithInfo emits it (batch-major, fp32) */
  const float* obs;        /* [B][T][D]   */
  const float* obs_next;   /* [B][1][D]   */
  const float* actions;    /* [B][T][A]   */
  const float* rewards;    /* [B][T]      */
  const float* dones;      /* [B][T]      */
  const float* behave;     /* [B][T][2A]  */
  const float* h0;         /* [L][B][H]  onetime_infos[0] layer-major */
  const float* c0;         /* [L][B][H]  onetime_infos[1]              */
  /* parameters */
  float* lstm; float* actor; float* critic;
  const float* ref_lstm; const float* ref_actor;
  float* zf_sum; float* zf_sumsq; float* zf_count;     /* updated by ZAPPLY */
  const float* rzf_sum; const float* rzf_sumsq; const float* rzf_count;
  float zf_eps;
  /* Adam state over [head | lstm] for each optimizer */
  float* actor_m; float* actor_v; float* critic_m; float* critic_v;
  int* actor_step; int* critic_step;
  const float* hyper;                /* SMI_HYP_* */
  const float* gamma_tab; const float* lam_tab;   /* torch.pow tables, [T] */
  float gamma, gamma_H;
  double kl_target;
  float kl_cutoff_coeff, actor_max_norm, critic_max_norm, actor_wd, critic_wd;
  float beta1, beta2, adam_eps;
  /* outputs */
  float* stats;                      /* [SMI_ST_COUNT] */
  float* kl_record; int* kl_count; int kl_capacity;
  /* exchange buffers (all-reduced by a data-parallel caller) */
  double* moments;                   /* [3] advantage (sum, sumsq, n) */
  double* pstat;                     /* [SMI_RNN_PSTAT] policy sums   */
  float* xbuf;                       /* [smi_ppo_rnn_xbuf_floats]: actor grads [actor | lstm]
                                        then critic grads [critic | lstm]                    */
  double* zbuf;                      /* [5 + 2*D] value sums | ZFilter column sums            */
  /* device scratch, smi_ppo_rnn_scratch_bytes() */
  void* scratch; int64_t scratch_bytes;
  /* optional pixel stem (if_pixel_input, ppo_net.py:137-141,268-275): the
   * LSTM input is [zfilter(low_dim) | CNN(camera0/255)] (D + cnn_feat wide);
   * cnn_feat == 0 disables it.  With it, `lstm` / `ref_lstm` point at the
   * joint stem buffer [lstm (in = D + cnn_feat) | cnn (smi_cnn_param_count)],
   * and the Adam state / xbuf segments are [head | lstm | cnn]. */
  int pix_c, pix_h, pix_w, cnn_feat;
  const uint8_t* pixels;        /* [B][T][C][H][W] uint8 (obs['pixel']['camera0'])      */
  const uint8_t* pixels_next;   /* [B][1][C][H][W] uint8 (obs_next['pixel']['camera0']) */
  /* optional (NULL: not written), filled by PREP: the windowed advantages as the
     policy epochs use them (normalised over all B_global*E windows when
     norm_adv, ppo.py:402-405) and the returns, both [B][E] batch-major */
  float* adv_out; float* ret_out;
  /* nn.LSTM num_layers (rnn_layer, ppo_net.py:146-149), 1..3 (0 = 1).  h0 / c0
     are then [rnn_layer][B][H] (onetime_infos[i].transpose(0, 1), ppo.py:508-509)
     and `lstm` / `ref_lstm` hold the layers one after another, each in
     nn.LSTM's order [W_ih | W_hh | b_ih | b_hh] (layer k >= 1: W_ih is 4H x H) */
  int rnn_layer;
  /* 0: PREP is issued after GAE on the same stream (GAE may run PREP's
     recurrence, see the phase table); != 0: PREP is independent of GAE (the
     caller runs it on another stream, before or beside GAE) */
  int prep_independent;
} smi_ppo_rnn_args;

#define SMI_RNN_PSTAT 16
int64_t smi_ppo_rnn_scratch_bytes(int B, int T, int horizon, int obs_dim, int rnn_hidden,
                                  int h1, int h2, int act_dim, int critic_h1, int critic_h2,
                                  int pix_c, int pix_h, int pix_w, int cnn_feat, int rnn_layer);
int64_t smi_ppo_rnn_xbuf_floats(int obs_dim, int rnn_hidden, int h1, int h2, int act_dim,
                                int critic_h1, int critic_h2, int pix_c, int pix_h, int pix_w,
                                int cnn_feat, int rnn_layer);
int64_t smi_lstm_param_count(int in_dim, int hidden);
int smi_ppo_rnn_phase(const smi_ppo_rnn_args* args, int phase, int epoch, void* stream);

/* LSTM sequence ops (nn.LSTM, one layer, batch_first semantics with
 * time-major buffers) — the building blocks of the phases above, exported for
 * tests and other callers:
 *   xproj [S][B][4H] = x W_ih^T + b_ih   (smi_linear_forward)
 *   forward: gates = xproj[t] + h_{t-1} W_hh^T + b_hh; c,h updates (i,f,g,o);
 *            hbuf[0] = h0, hbuf[t+1] = h_t ([S+1][B][H]); cbuf likewise and
 *            gates_act [S][B][4H] (activated) when non-NULL.
 *   backward: dgates [S][B][4H] from dh [S][B][H] (dL/dh_t from the heads),
 *            given gates_act and cbuf of the forward (BPTT through c and h). */
int smi_lstm_forward(const float* xproj, const float* w_hh, const float* b_hh,
                     const float* h0, const float* c0, int S, int B, int H,
                     float* hbuf, float* cbuf, float* gates_act, void* stream);
int smi_lstm_backward(const float* dh, const float* gates_act, const float* cbuf,
                      const float* w_hh, int S, int B, int H, float* dgates, void* stream);
/* forward over the raw inputs x [S][B] rows of ldx floats (din <= ldx used),
 * the input projection x W_ih^T + b_ih fused into the recurrence launch where
 * it fits (din <= 64, H <= 104), else the xproj GEMM and smi_lstm_forward's
 * recurrence; outputs as smi_lstm_forward.  Same semantics as nn.LSTM's layer
 * 0 (ppo_net.py:146-149: the policy / critic stem's rnn_stem). */
int smi_lstm_forward_x(const float* x, int64_t ldx, int din, const float* w_ih,
                       const float* b_ih, const float* w_hh, const float* b_hh,
                       const float* h0, const float* c0, int S, int B, int H, float* hbuf,
                       float* cbuf, float* gates_act, float* xproj_scratch, void* stream);

/* Pixel stem: CNNStemNetwork (builders.py:8-33) on obs/255 (ppo_net.py:368-375)
 *   conv 8x8/4 (C->16) -> ReLU -> conv 4x4/2 (16->32) -> ReLU -> Flatten -> Linear(F) -> ReLU
 * Flat parameters [conv1.w (16,C,8,8) | conv1.b | conv2.w (32,16,4,4) | conv2.b |
 * fc.w (F, 32*H2*W2) | fc.b].  Built for C == 3, W % 4 == 0 (84x84 cameras).
 * Images are uint8, 16-byte aligned; activation row n = t*B + b reads
 * pix[b][t] (t < T) or pix_next[b] (t == T) — a plain batch is B = rows, T = 1.
 *   forward: a1 [rows][16][H1*W1] (optional, needed by backward), a2 [rows][32*H2*W2],
 *            feat[n*ldf + f] = ReLU output.
 *   backward: dz = gradient at the Linear pre-activation (ReLU mask applied,
 *            row stride lddz); writes (not accumulates) the flat gradient. */
int64_t smi_cnn_param_count(int C, int H, int W, int F);
int64_t smi_cnn_scratch_bytes(int64_t rows, int C, int H, int W, int F);
int smi_cnn_forward(const float* params, const uint8_t* pix, const uint8_t* pix_next, int64_t B,
                    int64_t T, int64_t rows, int C, int H, int W, int F, float* a1, float* a2,
                    float* feat, int64_t ldf, void* stream);
int smi_cnn_backward(const float* params, const uint8_t* pix, const uint8_t* pix_next, int64_t B,
                     int64_t T, int64_t rows, int C, int H, int W, int F, const float* a1,
                     const float* a2, const float* dz, int64_t lddz, float* grad, void* scratch,
                     int64_t scratch_bytes, void* stream);

/* running_sum += sum_in, running_sumsq += sumsq_in, count += rows — the
 * data-parallel z_update after the column statistics were all-reduced. */
int smi_zfilter_accumulate(const float* sum_in, const float* sumsq_in, int dim, float rows,
                           float* running_sum, float* running_sumsq, float* count,
                           void* stream);

/* ---------------------------------------------------------- Adam / clip */
/* Replaces torch.nn.utils.clip_grad_norm_ + torch.optim.Adam.step
 * (as called at ppo.py:243-247,348-352) on one flat parameter buffer:
 *   norm = ||grad||; coef = min(1, max_norm/(norm+1e-6)) (if max_norm > 0);
 *   g = coef*grad (+ wd*p); m = lerp(m, g, 1-b1); v = b2*v + (1-b2) g^2;
 *   p -= (lr/(1-b1^t)) * m / (sqrt(v)/sqrt(1-b2^t) + eps)
 * `*step` (device int) is incremented; lr read from lr_ptr (device).
 * If skip_flag != NULL and *skip_flag != 0 the update is skipped entirely.
 * norm_out (device, may be NULL) receives the pre-clip norm. */
int smi_adam_clip(float* params, const float* grad, float* m, float* v, int64_t n,
                  int* step, const float* lr_ptr, float beta1, float beta2,
                  float eps, float weight_decay, float max_norm, float clip_value,
                  const int* skip_flag, float* norm_out, void* stream);
/* clip_value > 0 first clamps every gradient entry to [-clip_value, clip_value]
 * (nnx.Module.clip_grad_value as called at ddpg.py:309,332; torchx is not
 * available — the build states it as torch.nn.utils.clip_grad_value_). */

/* ------------------------------------------------ dense layers (MFMA GEMM) */
/* The Linear layers of builders.py:35-84 (DDPG ActorNetworkX / CriticNetworkX)
 * and any head too large for the single-CU kernels, as LDS-tiled fp32 MFMA
 * GEMMs over row-major operands with explicit leading dimensions (so a layer
 * can write into a column block of a wider concat buffer):
 *   forward:          y[r][o] = act(b[o] + sum_i x[r][i] w[o][i])   act 0/1/2
 *   backward_input:   dx[r][i] = [relu_mask[r][i] > 0] * sum_o dy[r][o] w[o][i]
 *   backward_weight:  dw[o][i] (+)= sum_r dy[r][o] x[r][i];  db[o] (+)= sum_r dy[r][o]
 * w is [out][ldw] row-major (torch nn.Linear when ldw == in); a column block of a
 * wider weight (the action block of CriticNetworkX's concat layer) is addressed
 * by offsetting w and keeping ldw.  Deterministic (no atomics). */
int smi_linear_forward(const float* x, int64_t ldx, int rows, int in_dim, const float* w,
                       int64_t ldw, const float* b, int out_dim, int act, float* y, int64_t ldy,
                       void* stream);
int smi_linear_backward_input(const float* dy, int64_t ldg, int rows, int out_dim,
                              const float* w, int64_t ldw, int in_dim, const float* relu_mask,
                              int64_t ldm, float* dx, int64_t lddx, void* stream);
/* smi_linear_forward plus y[r][out_dim + j] = s[r*lds + j] for j < s_cols in
 * the same launch: CriticNetworkX's cat(relu(x W1^T + b1), action) input of
 * its second layer (ddpg_net's critic, ddpg.py:244-352 callers) written by one
 * launch instead of a forward and a column copy. */
int smi_linear_forward_cat(const float* x, int64_t ldx, int rows, int in_dim, const float* w,
                           int64_t ldw, const float* b, int out_dim, int act, float* y,
                           int64_t ldy, const float* s, int64_t lds, int s_cols, void* stream);
int smi_linear_backward_weight(const float* dy, int64_t ldg, int rows, int out_dim,
                               const float* x, int64_t ldx, int in_dim, float* dw, int64_t lddw,
                               float* db, int accumulate, void* stream);
/* Grouped weight gradients: smi_linear_backward_weight calls between
 * smi_dw_group_begin() and smi_dw_group_flush(stream) (row-major operands,
 * outputs <= 512 x 512, at most 6 per group) are queued and run as ONE launch
 * (workgroups dealt over every GEMM's tiles x split-K slabs) plus one
 * fixed-order reduce at the flush; the caller keeps their dY / X buffers
 * unchanged until then.  Calls that do not qualify launch immediately. */
int smi_dw_group_begin(void);
int smi_dw_group_flush(void* stream);

/* ------------------------------------------------------- DDPG loss pieces */
/* critic loss nn.MSELoss()(Q, y) (ddpg.py:306): loss = mean((Q-y)^2), dQ = 2(Q-y)/n */
int smi_mse_grad(const float* q, int64_t q_stride, const float* y, int64_t n, float* dq,
                 float* loss, void* stream);
/* actor loss -Q(s, mu(s)).mean() (ddpg.py:325-329): loss, dQ = -1/n */
int smi_neg_mean_grad(const float* q, int64_t q_stride, int64_t n, float* dq, float* loss,
                      void* stream);
/* dz = dy * (1 - y^2) for y = tanh(z) */
int smi_tanh_backward(const float* dy, int64_t ldg, const float* y, int64_t ldy, int64_t rows,
                      int cols, float* dz, int64_t ldz, void* stream);
/* dst[r][0:cols] = src[r][0:cols] (strided) — the action block of torch.cat((h, a), 1) */
int smi_copy_cols(const float* src, int64_t lds, int64_t rows, int cols, float* dst,
                  int64_t ldd, void* stream);
/* LayerNorm blocks of the DDPG networks with use_layernorm=True (builders.py:
 * 41-48, 65-75: Linear -> ReLU -> L.LayerNorm(1)); L.LayerNorm(1) is taken as
 * torch.nn.LayerNorm(n) over the last dimension (biased variance, eps inside
 * the square root, affine), n <= 1024.  forward: y = (x - mean) rstd gamma +
 * beta per row, mean / rstd [rows] saved for the backward.  backward: dx from
 * dy (relu_input != 0: zero where x <= 0, the ReLU before the norm), and
 * dgamma = sum_rows dy xhat, dbeta = sum_rows dy (overwritten; fixed order). */
int smi_layernorm_forward(const float* x, int64_t ldx, int64_t rows, int n, const float* gamma,
                          const float* beta, float eps, float* y, int64_t ldy, float* mean,
                          float* rstd, void* stream);
int smi_layernorm_backward(const float* dy, int64_t ldg, const float* x, int64_t ldx,
                           const float* mean, const float* rstd, const float* gamma, int64_t rows,
                           int n, int relu_input, float* dx, int64_t lddx, float* dgamma,
                           float* dbeta, void* stream);

/* Batched parameter-noise acting (ddpg_agent.py:134-151,172-173; param_noise.py:
 * 17-24, 63-70): n agents, each with its own perturbed actor.  Row i of x
 * ([n][ldx], in_dim used) goes through the parameter set at params + i *
 * pstride: Linear(in, h1)-ReLU-Linear(h1, h2)-ReLU-Linear(h2, out)-out_act
 * (0 none, 1 ReLU, 2 tanh: ActorNetworkX, builders.py:35-56, without
 * LayerNorm); offsets6 (host) = the float offsets of W1 b1 W2 b2 W3 b3 inside
 * one set.  One launch for all n agents; widths <= 1024 (else SMI_E_NOFIT). */
int smi_mlp3_forward_stacked(const float* params, int64_t pstride, const int64_t* offsets6,
                             int in_dim, int h1, int h2, int out_dim, int out_act, const float* x,
                             int64_t ldx, int n, float* y, int64_t ldy, void* stream);

/* Parameter publish (module_dict.py:22-35, parameter_server.py:40-55: the
 * state_dict D2H of ModuleDict.dumps): copy nbytes (multiple of 16, 16-byte
 * aligned) from device memory into PINNED host memory with a kernel on
 * `stream` (the publisher's side stream), so the caller's thread never waits
 * in a DMA copy call.  Fails when host_dst is not pinned, mapped memory. */
int smi_copy_to_host(void* host_dst, const void* src, int64_t nbytes, void* stream);
/* The publisher's snapshot (module_dict.py:22-35: every state_dict tensor of
 * the published modules): n device segments srcs[i] (16-byte aligned, nbytes[i]
 * a multiple of 4) copied to dst + dst_offsets[i] (16-byte aligned) in one
 * launch per 16 segments on `stream` (the learner's, stream-ordered after the
 * last update).  srcs / dst_offsets / nbytes are host arrays. */
int smi_copy_gather(void* dst, const void* const* srcs, const int64_t* dst_offsets,
                    const int64_t* nbytes, int n, void* stream);
/* target <- tau*src + (1-tau)*target (soft target update, ddpg.py:409-417) */
int smi_soft_update(float* target, const float* src, int64_t n, float tau, void* stream);
/* action_norm, rewards, Q_target, Q_policy means of ddpg.py:335-345 -> stats4 */
int smi_ddpg_stats(const float* actions, int64_t lda, int act_dim, const float* rewards,
                   int64_t rs, const float* y, const float* q, int64_t qs, int64_t n,
                   float* stats4, void* stream);

/* ------------------------------------------------------ DDPG n-step target */
/* Replaces the target of DDPGLearner._optimize (surreal/learner/ddpg.py:279-283):
 *   y = r + gamma_n * q_next * (1 - done); with twin critics y = min(y, y2). */
int smi_ddpg_target(const float* rewards, const float* dones, const float* q_next,
                    const float* q_next2, int64_t n, float gamma_n, float* y,
                    void* stream);

/* ----------------------------------------- CPython-exact uniform sampling */
/* Replaces UniformReplay.sample's index draw
 * (surreal/replay/uniform_replay.py:43-47):
 *   [random.randint(0, n-1) for _ in range(batch)]
 * bit-exact with CPython's MT19937 (random.seed(int) init_by_array seeding,
 * _randbelow = getrandbits(k) with rejection).  The 624-word state lives in
 * device memory: state[0..623] words, state[624] = position.
 * smi_mt_seed runs on the HOST (it fills a host buffer of 625 uint32). */
int smi_mt_seed(uint64_t seed, uint32_t* host_state625);
int smi_mt_randint_host(uint32_t* host_state625, int64_t n, int64_t batch,
                        int64_t* out);
/* n must be in [1, 2^32 - 1]. */
int smi_mt_randint(uint32_t* dev_state625, int64_t n, int64_t batch,
                   int64_t* out_indices, void* stream);

/* Replay gather: out[i][:] = table[idx[i]][:] for `cols` floats per row. */
int smi_gather_rows(const float* table, int64_t cols, const int64_t* idx,
                    int64_t batch, float* out, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* SURREAL_MI_H */
