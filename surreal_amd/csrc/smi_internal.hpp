// smi_internal.hpp — host-side plumbing shared by the .hip translation units:
// error state for smi_last_error() and launch checking.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/surreal_mi.h"

namespace smi {

int set_error(int code, const char* msg);

// Optional per-launch HIP-event timing of the MFMA kernels (smi_kernel_timing):
// each launch records (class, algorithmic flops, start/end events) on its own
// stream.  Off by default; bench.py turns it on over its timed region.
// Classes up to KT_CNN_BWD count algorithmic flops; the HBM-bound streaming
// classes after them count algorithmic bytes (SURVEY §8(d) per-unit figures).
enum { KT_GEMM_FWD = 0, KT_GEMM_DX, KT_GEMM_DW, KT_GEMM_REDUCE, KT_LSTM_FWD, KT_LSTM_BWD,
       KT_CNN_FWD, KT_CNN_BWD,
       KT_GAE, KT_POLICY_STATS, KT_POLICY_GRAD, KT_VALUE_ROWS, KT_ADAM, KT_ZF_TMAJOR,
       KT_COUNT };
bool ktime_on();
int ktime_begin(hipStream_t st);                       // returns a slot, -1 when off/full
void ktime_end(int slot, int cls, double flops, hipStream_t st);
// device workspace of the calling thread's current smi_context (or the default
// one of smi_set_workspace): capacity in floats, and its base for a request of
// nfloats (nullptr when it does not fit)
int64_t smi_workspace_floats();
float* workspace_f32(int64_t nfloats);
// keep the first nfloats of this thread's workspace out of later requests
// (0: release); workspace_f32 / smi_workspace_floats serve what lies above
void workspace_reserve(int64_t nfloats);
int launch_linear_fwd(const float* X, int64_t ldx, int M, int K, const float* W, int64_t ldw,
                      const float* b, int N, int act, float* Y, int64_t ldy, hipStream_t st,
                      const int* skip = nullptr);
int launch_linear_bwd_dx(const float* dY, int64_t ldg, int M, int N, const float* W, int64_t ldw,
                         int K, const float* mask, int64_t ldm, float* dX, int64_t lddx,
                         hipStream_t st, const int* skip = nullptr);
int launch_linear_bwd_dw(const float* dY, int64_t ldg, int M, int N, const float* X, int64_t ldx,
                         int K, float* dW, int64_t lddw, float* db, int accumulate,
                         hipStream_t st, const int* skip = nullptr);
int launch_linear_bwd_dw2(const float* dY, int64_t ldg, int M, int N, const float* X1,
                          int64_t ldx1, int K1, const float* X2, int64_t ldx2, int K2,
                          float* dW1, int64_t ld1, float* dW2, int64_t ld2, float* db1,
                          float* db2, hipStream_t st, const int* skip = nullptr);
// grouped weight gradients: between dw_group_begin() and dw_group_flush(st) the
// eligible launch_linear_bwd_dw / _dw2 calls are queued (their operands must
// stay unchanged until the flush) and then run as ONE launch + ONE reduce
int dw_group_begin();
int dw_group_flush(hipStream_t st);
// Optional epilogue task of an open group's reducer (one more reducer block):
//   lvpart  (non-null) the PPO log_var gradient lv_out[j] = exp(lv[j]) *
//           sum_i lvpart[i][j] over lv_nb row-block partials (ppo_net.py:29-46)
//   sq      (non-null) fp64 sums of squares of every value the reducer stored
//           (one per reducer block, then the task's own), *np = their count:
//           the clip_grad_norm_ partials of the optimizer's Adam launch
//   step / runs  (non-null) incremented once (the optimizer's step counter)
//   skip    device stop flag (the task is a no-op when set)
struct DwEpilogue {
  int on;
  double* sq; int* np;
  const float* lvpart; int lv_nb, lv_A; const float* lv; float* lv_out;
  int* step; int* runs;
  const int* skip;
};
int dw_group_epilogue(const DwEpilogue& x);
// an M x N weight gradient (bias column included in N) joins an open group
bool dw_group_takes(int M, int N);
// BR of the one-segment-per-workgroup BPTT form for (B, H), 0 when another form runs
int lstm_bwd_q_form(int B, int H, const float* w_hh);
// the BPTT's step inputs staged in LDS (lstm_bwd_q_body) when they fit kBwdStageMax
bool use_bwd_stage();
constexpr size_t kBwdStageMax = 120 * 1024;
// the LSTM BPTT (lstm_bwd_q form) and the weight gradients queued so far in the
// open dW group in one launch (linear_kernels.hip); SMI_E_NOFIT: run
// launch_lstm_bwd instead (nothing launched)
int launch_lstm_bwd_dw(const float* dh, const float* gates, const float* cbuf, const float* w_hh,
                       int S, int B, int H, float* dgates, hipStream_t st, const int* skip);
int check_launch(const char* what);

// Test-only fault injection (build variant 'fault', -DSMI_FAULT_INJECTION;
// tests/negative_controls.py): deliberate departures from the reference the
// parity checks must catch.  The product library has no such state: fault()
// is the constant 0 there and every branch on it compiles away.
enum { SMI_FAULT_NONE = 0,
       SMI_FAULT_CRITIC_ADAM_SKIP = 1,     // value phases never apply Adam
       SMI_FAULT_CRITIC_STEM_OMIT = 2,     // the stems left out of the critic optimizer
       SMI_FAULT_POLICY_EPOCH_SHORT = 3,   // the last policy epoch's update skipped
       SMI_FAULT_GAE_HORIZON = 4 };        // GAE windows one step shorter than the horizon
#ifdef SMI_FAULT_INJECTION
int fault();
#else
constexpr int fault() { return SMI_FAULT_NONE; }
#endif

#define RC_CHECK(x) do { const int rc_ = (x); if (rc_) return rc_; } while (0)

// ---- pixel stem (CNNStemNetwork, builders.py:8-33) -------------------------
// Flat parameter layout (torch Conv2d / Linear shapes, in module order):
// [conv1.weight (16,C,8,8) | conv1.bias (16) | conv2.weight (32,16,4,4) |
//  conv2.bias (32) | fc.weight (F, 32*H2*W2) | fc.bias (F)]
struct CnnGeom {
  int C, H, W, H1, W1, P1, H2, W2, P2, K1, flat, F;
  int64_t img;                                  // bytes per uint8 image
  int64_t oW1, ob1, oW2, ob2, oWf, obf, total;  // offsets (floats)
  int64_t nconv;                                // conv parameters = oWf
};
__host__ __device__ inline CnnGeom cnn_geom(int C, int H, int W, int F) {
  CnnGeom g;
  g.C = C; g.H = H; g.W = W; g.F = F;
  g.H1 = (H - 8) / 4 + 1; g.W1 = (W - 8) / 4 + 1; g.P1 = g.H1 * g.W1;
  g.H2 = (g.H1 - 4) / 2 + 1; g.W2 = (g.W1 - 4) / 2 + 1; g.P2 = g.H2 * g.W2;
  g.K1 = 64 * C; g.flat = 32 * g.P2;
  g.img = (int64_t)C * H * W;
  g.oW1 = 0; g.ob1 = 16 * (int64_t)g.K1; g.oW2 = g.ob1 + 16; g.ob2 = g.oW2 + 32 * 256;
  g.oWf = g.ob2 + 32; g.obf = g.oWf + (int64_t)F * g.flat; g.total = g.obf + F;
  g.nconv = g.oWf;
  return g;
}
// image of activation row n = t*B + b: t < T -> pix[b][t], else pix_next[b]
struct PixRows { const unsigned char* pix; const unsigned char* pix_next; int64_t B, T, img_bytes; };
constexpr int kCnnPartials = 512;               // max workgroups (partial slabs) of the backward
int cnn_bwd_grid(int64_t rows);
int cnn_forward(const float* prm, const PixRows& pr, int C, int H, int W, int F, int64_t rows,
                float* A1, float* A2, float* feat, int64_t ldf, hipStream_t st, const int* skip);
// dz: gradient at the Linear pre-activation (ReLU mask applied), rows x F
// (stride lddz); writes the full gradient (not accumulated) into grad; dA2
// (rows x flat) and part (cnn_bwd_grid(rows) x nconv) are scratch.
int cnn_backward(const float* prm, const PixRows& pr, int C, int H, int W, int F, int64_t rows,
                 const float* A1, const float* A2, const float* dz, int64_t lddz, float* grad,
                 float* dA2, float* part, hipStream_t st, const int* skip);
int launch_slab_reduce(const float* part, int S, int64_t n, float* out, hipStream_t st,
                       const int* skip);

// Opt a kernel in to > 64 KiB of dynamic LDS (gfx950 has 160 KiB per CU).
// Host-only attribute call: no allocation, no stream work (graph-capture safe).
template <typename K>
inline void allow_lds(K kernel, size_t bytes) {
  if (bytes > 64 * 1024)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}

// Number of workgroups of `kernel` resident on the whole device at once
// (occupancy x CUs): the grid of a grid-stride streaming kernel, so every
// workgroup runs in the first and only round (no tail round at 60 % fill).
template <typename K>
inline int resident_grid(K kernel, int threads, size_t lds) {
  int dev = 0, cus = 256, per = 1;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, reinterpret_cast<const void*>(kernel),
                                                     threads, lds);
  if (per < 1) per = 1;
  return cus * per;
}

int64_t fused_lds_bytes(int B, int D, int H1, int H2, int A, int cH1, int cH2);

int launch_critic_gae(const float* critic_params, int D, int H1, int H2, int use_zf,
                      const float* zf_sum, const float* zf_sumsq, const float* zf_count,
                      float zf_eps, const float* obs, const float* obs_next,
                      const float* rewards, const float* dones, int B, int T,
                      const float* gtab, const float* ltab, float gamma, float gamma_T,
                      float* values, float* adv, float* ret, hipStream_t stream);
int gae_windows_max_partials(int64_t B, int T);
int launch_gae_windows(const float* values, float* values_masked, const float* rewards, const float* dones, int64_t B,
                       int T, int H, const float* gtab, const float* ltab, float gamma,
                       float gamma_H, float* adv, float* ret, double* partials,
                       int* n_partials, hipStream_t stream);
int launch_ppo_fused(const smi_ppo_args* args, hipStream_t stream);
int64_t ppo_fused_max_params();
int64_t ppo_xbuf_floats(int D, int H1, int H2, int A, int cH1, int cH2, int mode);
int launch_ppo_epoch_grad(const smi_ppo_args* args, int epoch, hipStream_t stream);
int launch_ppo_epoch_apply(const smi_ppo_args* args, int epoch, hipStream_t stream);

int64_t ppo_rnn_scratch_bytes(int B, int T, int Hz, int D, int H, int L, int h1, int h2, int A, int c1,
                              int c2, int pc, int ph, int pw, int F);
int ppo_rnn_phase(const smi_ppo_rnn_args& a, int phase, int e, hipStream_t st);
// keep: cbuf / gates stored for steps t < keep only (0: every step)
int launch_lstm_fwd(const float* xproj, const float* w_hh, const float* b_hh, const float* h0,
                    const float* c0, int S, int B, int H, float* hbuf, float* cbuf, float* gates,
                    hipStream_t st, const int* skip, int keep = 0);
int launch_lstm_fwd_x(const float* x, int64_t ldx, int din, const float* w_ih, const float* b_ih,
                      const float* w_hh, const float* b_hh, const float* h0, const float* c0,
                      int S, int B, int H, float* hbuf, float* cbuf, float* gates,
                      hipStream_t st, const int* skip, int keep = 0);
int launch_lstm_bwd(const float* dh, const float* gates, const float* cbuf, const float* w_hh,
                    int S, int B, int H, float* dgates, hipStream_t st, const int* skip);

}  // namespace smi
