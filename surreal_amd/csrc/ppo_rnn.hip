// ppo_rnn.hip — PPOLearner._optimize with the LSTM policy (if_rnn_policy;
// surreal/learner/ppo.py:487-586 and the RNN branch of _gae_and_return,
// ppo.py:389-406) as a fixed sequence of device phases (see surreal_mi.h).
//
// Rows of every activation are time-major, n = t*B + b (t < S), so the LSTM
// input projection, the heads and all weight gradients are plain GEMMs over
// contiguous matrices; per-row loss kernels map n back to the batch-major
// inputs.  Data-dependent control (KL early stop, adapt penalty branch) is a
// device flag that turns later phases into no-ops: the host issues the same
// launches on every call and every rank, and never waits for the device.
#include <stdlib.h>
#include "smi_device.hpp"
#include "smi_internal.hpp"
#include "pol_rows.hpp"
#include "lstm_cell.hpp"

namespace smi {

int launch_lstm_bwd(const float* dh, const float* gates, const float* cbuf, const float* w_hh,
                    int S, int B, int H, float* dgates, hipStream_t st, const int* skip);
bool lstm_fwd_x_dual_fits(int B0, int B1, int S, int H, int din);
int launch_lstm_fwd_x_dual(const LstmFwdArgs& a0, const LstmFwdArgs& a1, hipStream_t st);
int launch_gae_windows(const float* values, float* values_masked, const float* rewards,
                       const float* dones, int64_t B, int T, int H, const float* gtab,
                       const float* ltab, float gamma, float gamma_H, float* adv, float* ret,
                       double* partials, int* n_partials, hipStream_t stream);

// ----------------------------------------------------------------- layout
// final sums (fstat, double): value statistics of the last value epoch, then
// the ZFilter column sums of obs_iter
enum { FS_SE = 0, FS_D, FS_D2, FS_R, FS_R2, FS_Z = 5 };

struct RnnDims {
  int B, T, Hz, E, S1, D, H, G4, A, h1, h2, c1, c2;
  int L;                              // LSTM layers (nn.LSTM num_layers = rnn_layer)
  int64_t nL0, nLk;                   // parameters of layer 0 / of each layer above it
  int F, Din;                         // pixel features (0: no CNN stem), LSTM input D + F
  int Hin;                            // head input width: H (LSTM) or Din (H == 0: MLP policy)
  int ldx;                            // row stride of the stem input Xz / Xr: Din rounded up to
                                      // 4 (16-byte rows; the padding columns stay zero)
  int Hld;                            // row stride of the head input: H, or ldx (MLP policy)
  int64_t NE, NG;
  int64_t nA_head, nC_head, nL, nCnn, nS;   // parameter counts; stem = [lstm | cnn]
  MlpLayout LA, LC;
  CnnGeom G;
};

__host__ __device__ inline RnnDims rnn_dims(int B, int T, int Hz, int D, int H, int h1, int h2,
                                            int A, int c1, int c2, int pc = 0, int ph = 0,
                                            int pw = 0, int F = 0, int L = 1) {
  RnnDims d;
  d.L = L > 1 ? L : 1;
  d.F = F > 0 ? F : 0; d.Din = D + d.F;
  d.G = cnn_geom(pc, ph, pw, d.F);
  d.nCnn = d.F > 0 ? d.G.total : 0;
  d.B = B; d.T = T; d.Hz = Hz; d.E = T - Hz + 1; d.S1 = T + 1; d.D = D; d.H = H; d.G4 = 4 * H;
  d.A = A; d.h1 = h1; d.h2 = h2; d.c1 = c1; d.c2 = c2;
  d.NE = (int64_t)d.E * B; d.NG = (int64_t)d.S1 * B;
  d.Hin = H > 0 ? H : d.Din;
  d.ldx = (d.Din + 3) & ~3;
  d.Hld = H > 0 ? H : d.ldx;
  d.LA = mlp_layout(d.Hin, h1, h2, A, 1);
  d.LC = mlp_layout(d.Hin, c1, c2, 1, 0);
  d.nA_head = d.LA.fcount; d.nC_head = d.LC.fcount;
  // nn.LSTM parameter order per layer: W_ih, W_hh, b_ih, b_hh (layer k >= 1 reads
  // layer k-1's h, so its W_ih is 4H x H)
  d.nL0 = H > 0 ? (int64_t)4 * H * d.Din + (int64_t)4 * H * H + 8 * (int64_t)H : 0;
  d.nLk = H > 0 ? (int64_t)8 * H * H + 8 * (int64_t)H : 0;
  d.nL = d.nL0 + (d.L - 1) * d.nLk;
  d.nS = d.nL + d.nCnn;
  return d;
}

// scratch carve (floats, 64-float aligned regions)
struct RnnScratch {
  float *Xz, *Xr, *xproj, *hbuf, *cbuf, *gates, *HA1, *HA2, *OUT, *dOUT, *dH1, *dH2, *dh, *dgates;
  // the PREP phase's own copies (it may run on a second stream beside GAE)
  float *xprojR, *hbufR, *HA1R, *HA2R, *A2R;
  // W1^T | W2^T of the head a phase's fused forward wrote for its backward
  float *wT;
  float *values, *adv, *ret, *refmu, *lvpart;
  // time-major per-row inputs of the row kernels, packed once per learn,
  // field-major within blocks of 64 rows: rowin[rin_idx(W, n, f)], f =
  // {actions (A) | behave mu, sigma (2A) | raw advantage | behaviour
  // likelihood | KL(ref || behaviour) row term}, n = t*B + b;
  // ret_tm[n] the window return
  float *rowin, *ret_tm;
  float *A1, *A2, *dA2, *dF, *cpart;        // pixel stem (empty without one)
  double *part, *gaepart;
  int* ci; float* cf;
  int64_t total_floats;
};

static inline int64_t al64(int64_t n) { return (n + 63) & ~(int64_t)63; }
__host__ __device__ inline int rnn_nblk(int64_t rows, int nt = kWG) {
  // at most 1024 four-wave blocks' worth of waves (4096 one-wave blocks)
  const int64_t cap = (int64_t)1024 * kWG / nt;
  const int64_t b = (rows + nt - 1) / nt;
  return (int)(b < cap ? (b < 1 ? 1 : b) : cap);
}
// per-row loss kernels (a thread per row, ~100 dependent VALU / transcendental
// ops each): one-wave blocks so the rows of a C3 batch (21504) spread over
// 336 CUs' worth of blocks instead of 84 four-wave blocks
constexpr int kRowNT = 64;

int head_bwd_blocks(int64_t rows);
// doubles of s.part: 65536, or the value statistics' five per head workgroup
static int64_t part_doubles(const RnnDims& d) {
  const int64_t v = 5 * (int64_t)head_bwd_blocks(d.NE);
  return v > 65536 ? v : 65536;
}
// the last value epoch's statistics from the critic head forward's epilogue
// (SMI_VALUE_STATS_HEAD=0: value_rows_kernel; A/B knob)
static bool use_value_stats_head() {
  static const bool on = [] { const char* e = getenv("SMI_VALUE_STATS_HEAD"); return !(e && e[0] == '0'); }();
  return on;
}

static RnnScratch rnn_scratch(const RnnDims& d, void* base) {
  RnnScratch s{};
  float* p = static_cast<float*>(base);
  int64_t o = 0;
  auto take = [&](int64_t n) { float* r = p ? p + o : nullptr; o += al64(n); return r; };
  const int hmax1 = d.h1 > d.c1 ? d.h1 : d.c1, hmax2 = d.h2 > d.c2 ? d.h2 : d.c2;
  s.Xz = take(d.NG * d.ldx);
  s.Xr = take(d.NE * d.ldx);
  s.xproj = take(d.NG * d.G4);
  s.hbuf = take((int64_t)d.L * (d.S1 + 1) * d.B * d.H);     // per layer (see hbuf_of)
  s.cbuf = take((int64_t)d.L * (d.E + 1) * d.B * d.H);
  s.gates = take((int64_t)d.L * d.NE * d.G4);
  s.HA1 = take(d.NG * hmax1);
  s.HA2 = take(d.NG * hmax2);
  s.OUT = take(d.NG * (d.A > 1 ? d.A : 1));
  s.dOUT = take(d.NE * (d.A > 1 ? d.A : 1));
  s.dH1 = take(d.NE * hmax1);
  s.dH2 = take(d.NE * hmax2);
  s.dh = take(d.NE * d.H);
  s.dgates = take((int64_t)d.L * d.NE * d.G4);
  s.values = take((int64_t)d.B * d.S1);
  s.adv = take(d.NE);
  s.ret = take(d.NE);
  s.refmu = take(d.NE * d.A);
  s.rowin = take(((d.NE + 63) & ~(int64_t)63) * row_w(d.A));
  s.ret_tm = take(d.NE);
  s.lvpart = take((int64_t)4096 * d.A);
  const bool px = d.F > 0;
  s.A1 = take(px ? d.NE * 16 * d.G.P1 : 0);
  s.A2 = take(px ? d.NG * d.G.flat : 0);
  s.xprojR = take(d.NE * d.G4);
  s.hbufR = take((int64_t)d.L * (d.S1 + 1) * d.B * d.H);
  s.HA1R = take(d.NE * hmax1);
  s.HA2R = take(d.NE * hmax2);
  s.A2R = take(px ? d.NE * d.G.flat : 0);
  {
    const int64_t wa = (int64_t)d.Hin * d.h1 + (int64_t)d.h1 * d.h2;
    const int64_t wc = (int64_t)d.Hin * d.c1 + (int64_t)d.c1 * d.c2;
    s.wT = take(wa > wc ? wa : wc);
  }
  s.dA2 = take(px ? d.NE * d.G.flat : 0);
  s.dF = take(px ? d.NE * d.F : 0);
  s.cpart = take(px ? (int64_t)cnn_bwd_grid(d.NE) * d.G.nconv : 0);
  s.part = reinterpret_cast<double*>(take(2 * part_doubles(d)));   // >= 65536 doubles
  s.gaepart = reinterpret_cast<double*>(take(2 * 2 * 2048));
  s.ci = reinterpret_cast<int*>(take(CI_COUNT));
  s.cf = take(CF_COUNT);
  s.total_floats = o;
  return s;
}

// ------------------------------------------------------------ small kernels
// out[t][b][:] = zfilter(obs[b][t][:]) for t < T, out[T][b][:] = zfilter(obs_next[b][0][:]),
// for t < S (S <= T+1).  z_filter.py:59-79 (clamp +-5); use_zf == 0 copies.
// One wave per row (32-bit row index math once per row, not per element):
// lane j moves columns j, j + 64 of a D <= 128-wide row, so each load and
// store instruction covers one contiguous row.  A wave takes kZfRows rows per
// trip with every load issued before the first store (one row in flight per
// wave held the launch at ~0.24 of HBM at > 256 MB working sets).
constexpr int kZfRows = 8;
__global__ void __launch_bounds__(kWG)
zf_tmajor_kernel(const float* __restrict__ obs, const float* __restrict__ obs_next, int B, int T,
                 int S, int D, int use_zf, const float* zs, const float* zq, const float* zc,
                 float eps, float* __restrict__ out, int ldo) {
  if (D <= 0) return;                            // pixel-only: no low-dim columns
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* zm = sm;
  float* zd = sm + round4(D);
  if (use_zf) zfilter_colstats(zs, zq, zc, eps, D, zm, zd);
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int nrows = S * B;
  const int w0 = blockIdx.x * (kWG / 64) + (threadIdx.x >> 6), nw = gridDim.x * (kWG / 64);
  float m0 = 0.f, d0 = 1.f, m1 = 0.f, d1 = 1.f;
  if (use_zf) {
    if (lane < D) { m0 = zm[lane]; d0 = zd[lane]; }
    if (lane + 64 < D) { m1 = zm[lane + 64]; d1 = zd[lane + 64]; }
  }
  if ((D & 1) == 0 && (ldo & 1) == 0 && (reinterpret_cast<uintptr_t>(obs) & 7) == 0 &&
      (reinterpret_cast<uintptr_t>(obs_next) & 7) == 0 && (reinterpret_cast<uintptr_t>(out) & 7) == 0) {
    // even widths: 8-byte lanes, floor(128 / D) rows per load instruction
    // (D = 42: three rows on 63 lanes instead of one row on 42)
    const int D2 = D >> 1, rpi = 64 / D2;
    const int lr = lane / D2, lc = lane - lr * D2;
    const bool lv = lr < rpi;
    const int cc = lv ? 2 * lc : 0;
    float2 zm2 = {0.f, 0.f}, zd2 = {1.f, 1.f};
    if (use_zf) { zm2 = float2{zm[cc], zm[cc + 1]}; zd2 = float2{zd[cc], zd[cc + 1]}; }
    const int rpt = kZfRows * rpi;                  // rows per wave and trip
    for (int row0 = w0 * rpt; row0 < nrows; row0 += nw * rpt) {
      float2 v[kZfRows];
#pragma unroll
      for (int j = 0; j < kZfRows; ++j) {
        const int row = min(row0 + j * rpi + (lv ? lr : 0), nrows - 1);
        const int t = row / B, b = row - t * B;
        const float* src = t < T ? obs + ((int64_t)b * T + t) * D : obs_next + (int64_t)b * D;
        v[j] = *reinterpret_cast<const float2*>(src + cc);
      }
#pragma unroll
      for (int j = 0; j < kZfRows; ++j) {
        const int row = row0 + j * rpi + lr;
        if (!lv || row >= nrows) continue;
        float2 o = v[j];
        if (use_zf) {
          o.x = fminf(fmaxf((o.x - zm2.x) / zd2.x, -5.f), 5.f);
          o.y = fminf(fmaxf((o.y - zm2.y) / zd2.y, -5.f), 5.f);
        }
        *reinterpret_cast<float2*>(out + (int64_t)row * ldo + cc) = o;
      }
    }
    return;
  }
  const int c0 = lane < D ? lane : D - 1;               // clamped: unconditional loads
  const int c1 = lane + 64 < D ? lane + 64 : D - 1;
  const bool two = D > 64;
  for (int row0 = w0 * kZfRows; row0 < nrows; row0 += nw * kZfRows) {
    float v0[kZfRows], v1[kZfRows];
#pragma unroll
    for (int j = 0; j < kZfRows; ++j) {
      const int row = min(row0 + j, nrows - 1);
      const int t = row / B, b = row - t * B;
      const float* src = t < T ? obs + ((int64_t)b * T + t) * D : obs_next + (int64_t)b * D;
      v0[j] = src[c0];
      v1[j] = two ? src[c1] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < kZfRows; ++j) {
      const int row = row0 + j;
      if (row >= nrows) break;
      float* dst = out + (int64_t)row * ldo;
      if (lane < D) {
        float v = v0[j];
        if (use_zf) v = fminf(fmaxf((v - m0) / d0, -5.f), 5.f);
        dst[lane] = v;
      }
      if (lane + 64 < D) {
        float v = v1[j];
        if (use_zf) v = fminf(fmaxf((v - m1) / d1, -5.f), 5.f);
        dst[lane + 64] = v;
      }
    }
  }
}

// The same transform as a tile transpose through LDS (even D <= 128, 8-byte
// aligned rows): a workgroup takes kZfSeg segments, reads each one's S rows as
// ONE contiguous run (obs[b][0..T-1] is contiguous; the t = T row comes from
// obs_next) and writes, for every step t, the kZfSeg consecutive output rows
// t*B + b0 .. (contiguous too).  The row-per-wave kernel above reads 168-byte
// rows 4.4 KB apart: partial cache lines on every row, 0.42 of HBM at > 256 MB.
constexpr int kZfSeg = 8;
__global__ void __launch_bounds__(kWG)
zf_tile_kernel(const float* __restrict__ obs, const float* __restrict__ obs_next, int B, int T,
               int S, int D, int use_zf, const float* zs, const float* zq, const float* zc,
               float eps, float* __restrict__ out, int ldo) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* zm = sm;                                  // [round4(D)]
  float* zd = sm + round4(D);
  float* tile = sm + 2 * round4(D);                // [kZfSeg][S][D]
  if (use_zf) zfilter_colstats(zs, zq, zc, eps, D, zm, zd);
  const int b0 = blockIdx.x * kZfSeg;
  const int nseg = min(kZfSeg, B - b0);
  const int D2 = D >> 1, ST = min(S, T);
  // phase 1: each segment's rows, contiguous in obs, as float2 runs; eight
  // loads in flight per thread before their LDS stores (one at a time left
  // the block latency-bound: 0.34 of HBM)
  {
    const int per = ST * D2;                        // float2 per segment from obs
    const int tot = nseg * per;
    float2* t2 = reinterpret_cast<float2*>(tile);
    const float2* o2 = reinterpret_cast<const float2*>(obs + (int64_t)b0 * T * D);
    for (int base = 0; base < tot; base += 8 * kWG) {
      float2 r[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int e = min(base + k * kWG + (int)threadIdx.x, tot - 1);
        const int bl = e / per, q = e - bl * per;
        r[k] = o2[(int64_t)bl * T * D2 + q];
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int e = base + k * kWG + threadIdx.x;
        if (e < tot) {
          const int bl = e / per, q = e - bl * per;
          t2[(int64_t)bl * S * D2 + q] = r[k];
        }
      }
    }
    if (S > T) {
      for (int e = threadIdx.x; e < nseg * D2; e += kWG) {
        const int bl = e / D2, c = e - bl * D2;
        t2[(int64_t)bl * S * D2 + T * D2 + c] =
            reinterpret_cast<const float2*>(obs_next + (int64_t)(b0 + bl) * D)[c];
      }
    }
  }
  __syncthreads();
  // phase 2: thread (bl, c2) writes column pair c2 of segment bl at every step
  const int bl = threadIdx.x / D2, c2 = threadIdx.x - bl * D2;
  if (bl >= nseg) return;
  float2 m = {0.f, 0.f}, dd = {1.f, 1.f};
  if (use_zf) { m = float2{zm[2 * c2], zm[2 * c2 + 1]}; dd = float2{zd[2 * c2], zd[2 * c2 + 1]}; }
  const float2* tp = reinterpret_cast<const float2*>(tile + (int64_t)bl * S * D) + c2;
  float* op = out + (int64_t)(b0 + bl) * ldo + 2 * c2;
  for (int t = 0; t < S; ++t) {
    float2 v = tp[t * D2];
    if (use_zf) {
      v.x = fminf(fmaxf((v.x - m.x) / dd.x, -5.f), 5.f);
      v.y = fminf(fmaxf((v.y - m.y) / dd.y, -5.f), 5.f);
    }
    *reinterpret_cast<float2*>(op + (int64_t)t * B * ldo) = v;
  }
}

// zf_tile_kernel with 16-byte accesses on both sides (16-byte aligned obs,
// obs_next and out, ldo % 4 == 0): the kZfSeg segments' obs rows are ONE
// contiguous run, copied to LDS as float4 (the float2 copy above issued half
// the bytes per load instruction); the output rows of a step are written as
// float4 column chunks (the last one 1-3 wide when D % 4 != 0), every chunk of
// every (step, segment) row spread over the workgroup's threads.  Same
// arithmetic per element as the kernels above.
__global__ void __launch_bounds__(kWG)
zf_tile4_kernel(const float* __restrict__ obs, const float* __restrict__ obs_next, int B, int T,
                int S, int D, int use_zf, const float* zs, const float* zq, const float* zc,
                float eps, float* __restrict__ out, int ldo, int pad) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* zm = sm;                                  // [round4(D)]
  float* zd = sm + round4(D);
  float* tile = sm + 2 * round4(D);                // [kZfSeg][T][D], obs's own layout
  float* nxt = tile + round4(kZfSeg * T * D);      // [kZfSeg][D], the obs_next rows
  if (use_zf) zfilter_colstats(zs, zq, zc, eps, D, zm, zd);
  const int b0 = blockIdx.x * kZfSeg;
  const int nseg = min(kZfSeg, B - b0);
  {
    const int tot = nseg * T * D;                   // floats of the run (all T rows)
    const int tot4 = tot >> 2;
    const float4* src = reinterpret_cast<const float4*>(obs + (int64_t)b0 * T * D);
    float4* dst = reinterpret_cast<float4*>(tile);
    for (int base = 0; base < tot4; base += 8 * kWG) {
      float4 r[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) r[k] = src[min(base + k * kWG + (int)threadIdx.x, tot4 - 1)];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int e = base + k * kWG + threadIdx.x;
        if (e < tot4) dst[e] = r[k];
      }
    }
    for (int e = (tot4 << 2) + threadIdx.x; e < tot; e += kWG) tile[e] = obs[(int64_t)b0 * T * D + e];
    if (S > T) {
      const int tn = nseg * D, tn4 = tn >> 2;
      const float* nsrc = obs_next + (int64_t)b0 * D;
      for (int e = threadIdx.x; e < tn4; e += kWG)
        reinterpret_cast<float4*>(nxt)[e] = reinterpret_cast<const float4*>(nsrc)[e];
      for (int e = (tn4 << 2) + threadIdx.x; e < tn; e += kWG) nxt[e] = nsrc[e];
    }
  }
  __syncthreads();
  if (pad) {
    // ldo == round4(D) and columns D..ldo-1 are padding nobody reads: rows are
    // written whole, as float4 chunks, zeros in the padding, so a step's
    // kZfSeg output rows are one run of whole 128-byte lines (a row with an
    // 8-byte hole made every line a partial write)
    const int cpr = ldo >> 2, per_t = nseg * cpr;
    const int groups = kWG / per_t;
    const int g = threadIdx.x / per_t, r = threadIdx.x - g * per_t;
    if (g >= groups) return;
    const int bl = r / cpr, c = 4 * (r - bl * cpr);
    float zmv[4], zdv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      zmv[j] = use_zf && c + j < D ? zm[c + j] : 0.f;
      zdv[j] = use_zf && c + j < D ? zd[c + j] : 1.f;
    }
    const bool even = (D & 1) == 0;
    for (int t = g; t < S; t += groups) {
      const float* sp = t < T ? tile + ((int64_t)bl * T + t) * D + c : nxt + bl * D + c;
      float v[4];
      if (even) {
        const float2 lo = *reinterpret_cast<const float2*>(sp);
        const float2 hi = c + 2 < D ? *reinterpret_cast<const float2*>(sp + 2) : float2{0.f, 0.f};
        v[0] = lo.x; v[1] = lo.y; v[2] = hi.x; v[3] = hi.y;
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = c + j < D ? sp[j] : 0.f;
      }
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (use_zf && c + j < D) v[j] = fminf(fmaxf((v[j] - zmv[j]) / zdv[j], -5.f), 5.f);
      *reinterpret_cast<float4*>(out + ((int64_t)t * B + b0 + bl) * ldo + c) =
          float4{v[0], v[1], v[2], v[3]};
    }
    return;
  }
  if (D % 2 == 0 && D / 2 * kZfSeg <= kWG) {
    // even widths: zf_tile_kernel's phase 2 (thread = segment x column pair,
    // conflict-free 8-byte LDS reads, one float2 store per step)
    const int D2 = D >> 1;
    const int bl = threadIdx.x / D2, c2 = threadIdx.x - bl * D2;
    if (bl >= nseg) return;
    float2 m = {0.f, 0.f}, dd = {1.f, 1.f};
    if (use_zf) { m = float2{zm[2 * c2], zm[2 * c2 + 1]}; dd = float2{zd[2 * c2], zd[2 * c2 + 1]}; }
    const float2* tp = reinterpret_cast<const float2*>(tile + (int64_t)bl * T * D) + c2;
    float* op = out + (int64_t)(b0 + bl) * ldo + 2 * c2;
    for (int t = 0; t < S; ++t) {
      float2 v = t < T ? tp[t * D2] : reinterpret_cast<const float2*>(nxt + bl * D)[c2];
      if (use_zf) {
        v.x = fminf(fmaxf((v.x - m.x) / dd.x, -5.f), 5.f);
        v.y = fminf(fmaxf((v.y - m.y) / dd.y, -5.f), 5.f);
      }
      *reinterpret_cast<float2*>(op + (int64_t)t * B * ldo) = v;
    }
    return;
  }
  const int cpr = (D + 3) >> 2;                    // column chunks per row
  const int per_t = nseg * cpr;
  const int tot = S * per_t;
  for (int e = threadIdx.x; e < tot; e += kWG) {
    const int t = e / per_t, r = e - t * per_t;
    const int bl = r / cpr, k = r - bl * cpr;
    const int c = 4 * k, w = min(4, D - c);
    const float* sp = t < T ? tile + ((int64_t)bl * T + t) * D + c : nxt + bl * D + c;
    float v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v[j] = j < w ? sp[j] : 0.f;
      if (use_zf && j < w) v[j] = fminf(fmaxf((v[j] - zm[c + j]) / zd[c + j], -5.f), 5.f);
    }
    float* op = out + ((int64_t)t * B + b0 + bl) * ldo + c;
    if (w == 4) {
      *reinterpret_cast<float4*>(op) = float4{v[0], v[1], v[2], v[3]};
    } else if (w == 2) {
      *reinterpret_cast<float2*>(op) = float2{v[0], v[1]};
    } else {
      for (int j = 0; j < w; ++j) op[j] = v[j];
    }
  }
}

// zf_tile4_kernel's padded-row form as a resident grid looping over tiles,
// software-pipelined: tile i+1's obs run is loaded into registers (kZfNR
// float4 per thread) while tile i's rows are written from LDS, then stored to
// the other LDS buffer, so every workgroup keeps reads and writes in flight at
// once (the one-shot tile kernel alternated a read phase and a write phase)
constexpr int kZfNR = 10;
__global__ void __launch_bounds__(kWG)
zf_pipe_kernel(const float* __restrict__ obs, const float* __restrict__ obs_next, int B, int T,
               int S, int D, int use_zf, const float* zs, const float* zq, const float* zc,
               float eps, float* __restrict__ out, int ldo) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* zm = sm;
  float* zd = sm + round4(D);
  const int TD = T * D;
  const int tile_f = round4(kZfSeg * TD), buf_f = tile_f + round4(kZfSeg * D);
  float* buf0 = sm + 2 * round4(D);
  if (use_zf) zfilter_colstats(zs, zq, zc, eps, D, zm, zd);
  const int ntile = (B + kZfSeg - 1) / kZfSeg;
  const bool has_next = S > T;
  float4 r0, r1, r2, r3, r4, r5, r6, r7, r8, r9;   // kZfNR named registers (an
  float4 rn = {0.f, 0.f, 0.f, 0.f};                // array here went to scratch)
  static_assert(kZfNR == 10, "zf_pipe_kernel: ten staging registers");
// registers <- tile TL's obs run (and its obs_next rows)
#define ZF_LOAD(TL)                                                                          \
  do {                                                                                       \
    const int lb0 = (TL) * kZfSeg, lns = min(kZfSeg, B - lb0);                               \
    const int lt4 = (lns * TD) >> 2;                                                         \
    const float4* src = reinterpret_cast<const float4*>(obs + (int64_t)lb0 * TD);            \
    if (lt4 > 0) {                                                                           \
      const int tx = threadIdx.x, m = lt4 - 1;                                               \
      r0 = src[min(tx, m)]; r1 = src[min(tx + kWG, m)]; r2 = src[min(tx + 2 * kWG, m)];      \
      r3 = src[min(tx + 3 * kWG, m)]; r4 = src[min(tx + 4 * kWG, m)];                        \
      r5 = src[min(tx + 5 * kWG, m)]; r6 = src[min(tx + 6 * kWG, m)];                        \
      r7 = src[min(tx + 7 * kWG, m)]; r8 = src[min(tx + 8 * kWG, m)];                        \
      r9 = src[min(tx + 9 * kWG, m)];                                                        \
    }                                                                                        \
    const int ln4 = (lns * D) >> 2;                                                          \
    if (has_next && ln4 > 0)                                                                 \
      rn = reinterpret_cast<const float4*>(obs_next + (int64_t)lb0 * D)[min((int)threadIdx.x, ln4 - 1)]; \
  } while (0)
// registers (+ the few floats past the last whole float4) -> LDS buffer BUF
#define ZF_STASH(TL, BUF)                                                                    \
  do {                                                                                       \
    const int lb0 = (TL) * kZfSeg, lns = min(kZfSeg, B - lb0);                               \
    const int ltot = lns * TD, lt4 = ltot >> 2;                                              \
    float4* dst = reinterpret_cast<float4*>(BUF);                                            \
    const int tx = threadIdx.x;                                                              \
    if (tx < lt4) dst[tx] = r0;                                                              \
    if (tx + kWG < lt4) dst[tx + kWG] = r1;                                                  \
    if (tx + 2 * kWG < lt4) dst[tx + 2 * kWG] = r2;                                          \
    if (tx + 3 * kWG < lt4) dst[tx + 3 * kWG] = r3;                                          \
    if (tx + 4 * kWG < lt4) dst[tx + 4 * kWG] = r4;                                          \
    if (tx + 5 * kWG < lt4) dst[tx + 5 * kWG] = r5;                                          \
    if (tx + 6 * kWG < lt4) dst[tx + 6 * kWG] = r6;                                          \
    if (tx + 7 * kWG < lt4) dst[tx + 7 * kWG] = r7;                                          \
    if (tx + 8 * kWG < lt4) dst[tx + 8 * kWG] = r8;                                          \
    if (tx + 9 * kWG < lt4) dst[tx + 9 * kWG] = r9;                                          \
    for (int e = (lt4 << 2) + tx; e < ltot; e += kWG) (BUF)[e] = obs[(int64_t)lb0 * TD + e]; \
    if (has_next) {                                                                          \
      float* nb = (BUF) + tile_f;                                                            \
      const int tn = lns * D, tn4 = tn >> 2;                                                 \
      if (tx < tn4) reinterpret_cast<float4*>(nb)[tx] = rn;                                  \
      for (int e = (tn4 << 2) + tx; e < tn; e += kWG) nb[e] = obs_next[(int64_t)lb0 * D + e]; \
    }                                                                                        \
  } while (0)
  const int cpr = ldo >> 2, per_t = kZfSeg * cpr;
  const int groups = kWG / per_t;
  const int g = threadIdx.x / per_t, rr = threadIdx.x - g * per_t;
  const int bl = rr / cpr, c = 4 * (rr - bl * cpr);
  float zmv[4], zdv[4];
  __syncthreads();                                 // zm / zd
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    zmv[j] = use_zf && c + j < D ? zm[c + j] : 0.f;
    zdv[j] = use_zf && c + j < D ? zd[c + j] : 1.f;
  }
  const bool even = (D & 1) == 0;
  int tl = blockIdx.x;
  if (tl < ntile) { ZF_LOAD(tl); ZF_STASH(tl, buf0); }
  int cur = 0;
  for (; tl < ntile; tl += gridDim.x) {
    __syncthreads();                               // buffer `cur` complete
    const int nx = tl + gridDim.x;
    if (nx < ntile) ZF_LOAD(nx);                   // in flight behind the writes below
    float* buf = buf0 + cur * buf_f;
    const int b0 = tl * kZfSeg, nseg = min(kZfSeg, B - b0);
    if (g < groups && bl < nseg) {
      for (int t = g; t < S; t += groups) {
        const float* sp = t < T ? buf + (bl * T + t) * D + c : buf + tile_f + bl * D + c;
        float v[4];
        if (even) {
          const float2 lo = *reinterpret_cast<const float2*>(sp);
          const float2 hi = c + 2 < D ? *reinterpret_cast<const float2*>(sp + 2) : float2{0.f, 0.f};
          v[0] = lo.x; v[1] = lo.y; v[2] = hi.x; v[3] = hi.y;
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = c + j < D ? sp[j] : 0.f;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (use_zf && c + j < D) v[j] = fminf(fmaxf((v[j] - zmv[j]) / zdv[j], -5.f), 5.f);
        *reinterpret_cast<float4*>(out + ((int64_t)t * B + b0 + bl) * ldo + c) =
            float4{v[0], v[1], v[2], v[3]};
      }
    }
    cur ^= 1;
    if (nx < ntile) ZF_STASH(nx, buf0 + cur * buf_f);
  }
#undef ZF_LOAD
#undef ZF_STASH
}

// values[b][t] = vt[t*B + b]
__global__ void __launch_bounds__(kWG)
tmajor_to_bmajor_kernel(const float* __restrict__ vt, int S, int B, float* __restrict__ v,
                        int* ci, float* cf) {
  // the learn()'s device control state starts at zero (was rnn_init_kernel,
  // a launch of its own): nothing before this point of the GAE phase reads it
  if (blockIdx.x == 0 && ci && threadIdx.x < CI_COUNT) ci[threadIdx.x] = 0;
  if (blockIdx.x == 0 && cf && threadIdx.x < CF_COUNT) cf[threadIdx.x] = 0.f;
  const int64_t n = (int64_t)S * B;
  for (int64_t e = (int64_t)blockIdx.x * kWG + threadIdx.x; e < n; e += (int64_t)gridDim.x * kWG) {
    const int b = (int)(e / S), t = (int)(e - (int64_t)b * S);
    v[e] = vt[(int64_t)t * B + b];
  }
}

// fixed-order reduction of [nb][w] double partials -> out[w] (one workgroup).
// Column j is summed by a group of L lanes (L the largest power of two <= 64
// with w * L <= kWG, so a group never straddles a wave): lane l of the group
// adds partials l, l + L, ... in order, then a butterfly over the group.  (One
// wave per column left a 2 x 42-column ZFilter reduction 21 serial
// butterflies deep per wave: 29 us for 21.5 K doubles.)  cnt != null: also
// out[w] = n (the advantage count of the GAE moments)
__global__ void __launch_bounds__(kWG)
reduce_partials_kernel(const double* __restrict__ part, int nb, int w, double* out,
                       const int* skip, double* cnt, double n) {
  if (skip && skip[0] != 0) return;
  if (cnt && threadIdx.x == 0) cnt[0] = n;
  int L = 64;
  while (L > 1 && w * L > kWG) L >>= 1;
  const int j = threadIdx.x / L, l = threadIdx.x - j * L;
  for (int jj = j; jj < w; jj += kWG / L) {
    // four partials in flight per lane (independent sums, combined in order)
    double s4[4] = {0.0, 0.0, 0.0, 0.0};
    int i = l;
    // four of those steps' loads (16 partials) per round trip, added in the
    // steps' order (a column summed by few lanes had one trip per 4 partials)
    for (; i + 15 * L < nb; i += 16 * L) {
      double v[4][4];
#pragma unroll
      for (int it = 0; it < 4; ++it)
#pragma unroll
        for (int k = 0; k < 4; ++k) v[it][k] = part[(int64_t)(i + (4 * it + k) * L) * w + jj];
#pragma unroll
      for (int it = 0; it < 4; ++it)
#pragma unroll
        for (int k = 0; k < 4; ++k) s4[k] += v[it][k];
    }
    for (; i + 3 * L < nb; i += 4 * L) {
#pragma unroll
      for (int k = 0; k < 4; ++k) s4[k] += part[(int64_t)(i + k * L) * w + jj];
    }
    for (; i < nb; i += L) s4[0] += part[(int64_t)i * w + jj];
    double s = (s4[0] + s4[1]) + (s4[2] + s4[3]);
    for (int o = L >> 1; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if (l == 0) out[jj] = s;
  }
}

// optional export of the advantages as the epochs use them and the returns,
// both [B][E] batch-major (smi_ppo_rnn_args.adv_out / ret_out)
__global__ void __launch_bounds__(kWG)
adv_export_kernel(PolRowArgs a, float* __restrict__ adv_out, float* __restrict__ ret_out) {
  const int64_t n = (int64_t)a.B * a.E;
  const AdvNorm nadv(a);
  for (int64_t e = (int64_t)blockIdx.x * kWG + threadIdx.x; e < n; e += (int64_t)gridDim.x * kWG) {
    if (adv_out) adv_out[e] = nadv(a.adv[e]);
    if (ret_out) ret_out[e] = a.ret[e];
  }
}

// rowin / ret_tm from the batch-major inputs (once per learn), field-major in
// 64-row blocks: the per-row kernels of every epoch give a thread one row, so
// lane i reads field f of row n0 + i and one load instruction covers 64
// consecutive floats
// (a row-major 100-byte row per lane made every load instruction touch ~56
// cache lines: the row kernels waited on the texture addresser, PMC TA_BUSY)
// + each row's behaviour-policy terms (behave_terms: the reference means
// refmu of PREP and the reference std are fixed for the learn)
template <int AT>
__global__ void __launch_bounds__(kWG)
row_pack_kernel(PolRowArgs a, float* __restrict__ rowin, float* __restrict__ ret_tm) {
  constexpr int AM = AT > 0 ? AT : 32;
  const int A = AT > 0 ? AT : a.A;
  float lrsig[AM], s02[AM];                        // PolStatsCols' reference-std terms
#pragma unroll
  for (int j = 0; j < (AT > 0 ? AT : A); ++j) {
    const float rsig = expf(a.ref_lv[j]);
    s02[j] = rsig * rsig;
    lrsig[j] = logf(rsig);
  }
  const int64_t N = (int64_t)a.E * a.B;
  const int W = row_w(A);
  for (int64_t n = (int64_t)blockIdx.x * kWG + threadIdx.x; n < N; n += (int64_t)gridDim.x * kWG) {
    const int t = (int)(n / a.B), b = (int)(n - (int64_t)t * a.B);
    const int64_t src = (int64_t)b * a.T + t;
    const float* acp = a.actions + src * A;
    const float* bh = a.behave + src * 2 * A;
    float ac[AM], bmu[AM], bsd[AM], rm[AM];
#pragma unroll
    for (int j = 0; j < (AT > 0 ? AT : A); ++j) {
      ac[j] = acp[j];
      bmu[j] = bh[j];
      bsd[j] = bh[A + j];
      rm[j] = a.refmu[n * A + j];
    }
#pragma unroll
    for (int j = 0; j < (AT > 0 ? AT : A); ++j) {
      rowin[rin_idx(W, n, j)] = ac[j];
      rowin[rin_idx(W, n, A + j)] = bmu[j];
      rowin[rin_idx(W, n, 2 * A + j)] = bsd[j];
    }
    rowin[rin_idx(W, n, rin_adv(A))] = a.adv[(int64_t)b * a.E + t];
    float bl, rbd;
    behave_terms<AT>(ac, bmu, bsd, rm, lrsig, s02, A, a.c_ll, bl, rbd);
    rowin[rin_idx(W, n, rin_bl(A))] = bl;
    rowin[rin_idx(W, n, rin_rbd(A))] = rbd;
    ret_tm[n] = a.ret[(int64_t)b * a.E + t];
  }
}

static void launch_row_pack(int A, int64_t rows, const PolRowArgs& p, float* rowin, float* ret_tm,
                            hipStream_t st) {
  const int g = (int)std::max<int64_t>(1, std::min<int64_t>(1024, (rows + kWG - 1) / kWG));
  switch (A) {
#define RP(K) case K: hipLaunchKernelGGL(row_pack_kernel<K>, dim3(g), dim3(kWG), 0, st, p, rowin, ret_tm); break;
    RP(1) RP(2) RP(3) RP(4) RP(5) RP(6) RP(7) RP(8)
#undef RP
    default: hipLaunchKernelGGL(row_pack_kernel<0>, dim3(g), dim3(kWG), 0, st, p, rowin, ret_tm); break;
  }
}

// forward statistics of the policy over the E*B rows (ppo.py:203-224,
// 262-284, 553-575)
// FUSE (clip mode): the same pass also writes the per-row gradient dz and the
// d/dstd block partials that policy_rows_grad_kernel would compute for this
// epoch (the clip surrogate's gradient needs no global statistic: weight 1/N,
// no KL term), bit-identically, so the gradient phase skips its row pass
template <int NT, int AT, bool FUSE>
__global__ void __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(1, AT > 0 ? 3 : 8)))
policy_rows_stats_kernel(PolRowArgs a) {
  constexpr int AM = AT > 0 ? AT : 32;
  __shared__ float ssig[32], slsig[32], srsig[32];
  __shared__ double scr[NT / 64][PS_N];
  __shared__ float gls[FUSE ? NT / 64 : 1][32];
  const int A = AT > 0 ? AT : a.A;
  const int64_t N = (int64_t)a.E * a.B;
  const int64_t n0 = (int64_t)blockIdx.x * NT + threadIdx.x, ns = (int64_t)gridDim.x * NT;
  // one row's inputs; with a compile-time action width the row loop runs two
  // alternating register sets, the next row's loads in flight behind this
  // row's arithmetic (clamped row index: always issued, so the waitcnt pass
  // waits for exactly the set it consumes)
  // (bl / rbd: the row's behaviour-policy terms, packed once per learn)
  struct RowIn { float m[AM], rm[AM], ac[AM], adv, ret, bl, rbd; };
  auto load_row = [&](RowIn& x, int64_t n) {
    ld_row<AT>(x.m, a.mu + n * A, A);
    ld_row<AT>(x.rm, a.refmu + n * A, A);
    ld_fields<AT>(x.ac, a.rowin, N, n, 0, A);
    x.adv = a.rowin[rin_idx(row_w(A), n, rin_adv(A))];
    x.bl = a.rowin[rin_idx(row_w(A), n, rin_bl(A))];
    x.rbd = a.rowin[rin_idx(row_w(A), n, rin_rbd(A))];
    x.ret = a.ret_tm[n];
  };
  // every load ahead of the first wait (as in pol_grad_weights): the stds'
  // log_vars (column threadIdx.x, A <= 32 < NT, clamped), the first row
  // (clamped), then the scalars with the skip flag — one round trip for all
  // (the flag, the log_vars, the clip range, the moments and the row had
  // waited one after the other)
  const int jc = min((int)threadIdx.x, A - 1);
  float lvj = a.lv[jc], rlvj = a.ref_lv[jc];
  [[maybe_unused]] RowIn X0, X1;
  if constexpr (AT > 0) load_row(X0, n0 < N ? n0 : N - 1);
  const int* zi = reinterpret_cast<const int*>(g_pol_zero);
  const double* mp = (a.norm_adv && a.moments) ? a.moments : g_pol_zero;
  int sk = *(a.skip ? a.skip : zi);
  float clip_lo = a.hyper[SMI_HYPX_CLIP_LO], clip_hi = a.hyper[SMI_HYPX_CLIP_HI];
  double mom[3] = {mp[0], mp[1], mp[2]};
  // (pinned together: left to their uses, the moments' loads sank into
  // AdvNorm's branch and the clip range's past it, a scalar round trip each)
  asm volatile("" : "+s"(sk), "+s"(clip_lo), "+s"(clip_hi));
  asm volatile("" : "+s"(mom[0]), "+s"(mom[1]), "+s"(mom[2]));
  asm volatile("" : "+v"(lvj));
  asm volatile("" : "+v"(rlvj));
  if (sk != 0) return;
  if ((int)threadIdx.x < A) {
    const int j = threadIdx.x;
    ssig[j] = expf(lvj);                     // builders.py:127 std = exp(log_var)
    slsig[j] = logf(ssig[j]);                // std0.log() of ppo_net.py:40
    srsig[j] = expf(rlvj);
  }
  __syncthreads();
  // per-column terms of the learner std (log-likelihood, KL(ref || learner))
  // and the reference std (KL(ref || behaviour)), hoisted out of the row loop;
  // divisions by them become multiplications by hoisted reciprocals (one
  // rounding more per term: row_loglik_r)
  float sig[AM], isig[AM], lsig[AM], lkl[AM], s02[AM], iden2[AM], lrsig[AM];
#pragma unroll
  for (int j = 0; j < (AT > 0 ? AT : A); ++j) {
    sig[j] = ssig[j]; lsig[j] = slsig[j];
    const float rsig = srsig[j];
    isig[j] = 1.f / sig[j];
    lkl[j] = logf(sig[j] / rsig);               // row_kl(rm, rsig, m, sig)'s per-column terms
    s02[j] = rsig * rsig;
    iden2[j] = 1.f / (2.f * (sig[j] * sig[j]));
    lrsig[j] = logf(rsig);
  }
  double acc[PS_N];
#pragma unroll
  for (int k = 0; k < PS_N; ++k) acc[k] = 0.0;
  float glv[AM];
  if constexpr (FUSE) {
#pragma unroll
    for (int j = 0; j < (AT > 0 ? AT : A); ++j) glv[j] = 0.f;
  }
  const AdvNorm nadv(a, mom);
  auto row = [&](const RowIn& x, int64_t n) {
    const float* m = x.m;
    const float* rm = x.rm;
    const float* ac = x.ac;
    const float av = nadv(x.adv);
    const float ex = expf(row_loglik_r<AT>(ac, m, isig, lsig, A, a.c_ll));
    const float lp = fmaxf(ex, 1e-5f);
    const float bl = x.bl;
    acc[PS_KL] += (double)row_kl_cc<AT>(rm, m, lkl, s02, iden2, A);
    // both modes add into fixed accumulators (adapt adds an exact 0 to the
    // clip sum): merged branches had indexed acc[] by mode, i.e. from scratch
    float t_surr, t_clip;
    if (a.mode == 0) {
      const float ratio = lp / bl;
      const float cr = fminf(fmaxf(ratio, clip_lo), clip_hi);
      const float surr = -ratio * av, csur = -cr * av;
      t_surr = surr;
      t_clip = fmaxf(surr, csur);
    } else {
      t_surr = av * (lp / fmaxf(bl, 1e-2f));
      t_clip = 0.f;
    }
    acc[PS_SURR] += (double)t_surr;
    acc[PS_CLIP] += (double)t_clip;
    acc[PS_ISW] += (double)(lp / (bl + 1e-4f));
    acc[PS_BL] += (double)bl;
    acc[PS_RBD] += (double)x.rbd;
    acc[PS_RET] += (double)x.ret;
    if constexpr (FUSE) {          // policy_rows_grad_kernel's clip branch, weight a.invN
      const float ratio = lp / bl;
      const float cr = fminf(fmaxf(ratio, clip_lo), clip_hi);
      const float surr = -ratio * av, csur = -cr * av;
      const float g_lp = ((surr >= csur) ? -(a.invN * av) : 0.f) / bl;
      const float g_ll = (ex >= 1e-5f) ? g_lp * ex : 0.f;
      float dz[AM];
#pragma unroll
      for (int j = 0; j < (AT > 0 ? AT : A); ++j) {
        const float i1 = isig[j];
        const float u = (ac[j] - m[j]) * i1;
        const float gmu = g_ll * (u * i1);
        const float gsd = g_ll * (u * u * i1 - i1);
        glv[j] += gsd;
        dz[j] = gmu * (1.f - m[j] * m[j]);
      }
      st_row<AT>(a.dz + n * A, dz, A);
    }
  };
  if constexpr (AT > 0) {
    for (int64_t n = n0; n < N; n += 2 * ns) {
      load_row(X1, min(n + ns, N - 1));
      row(X0, n);
      if (n + ns >= N) break;
      load_row(X0, min(n + 2 * ns, N - 1));
      row(X1, n + ns);
    }
  } else {
    for (int64_t n = n0; n < N; n += ns) {
      RowIn X;
      load_row(X, n);
      row(X, n);
    }
  }
  if constexpr (FUSE) {            // block partials of sum_rows d/dstd, as the grad kernel
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int j = 0; j < (AT > 0 ? AT : A); ++j) {
      const float sg = wave_sum(glv[j]);
      if (lane == 0) gls[wave][j] = sg;
    }
    __syncthreads();
    for (int j = threadIdx.x; j < A; j += NT) {
      float sg = 0.f;
      for (int w = 0; w < NT / 64; ++w) sg += gls[w][j];
      a.lvpart[(int64_t)blockIdx.x * A + j] = sg;
    }
  }
  // all PS_N sums at once: wave butterflies, one barrier, fixed wave order
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < PS_N; ++k) {
    const double v = wave_sum_d(acc[k]);
    if (lane == 0) scr[wave][k] = v;
  }
  __syncthreads();
  if (threadIdx.x < PS_N) {
    double t = 0.0;
#pragma unroll
    for (int w = 0; w < NT / 64; ++w) t += scr[w][threadIdx.x];
    a.part[(int64_t)blockIdx.x * PS_N + threadIdx.x] = t;
  }
}

// per-row gradient of the policy loss w.r.t. the tanh pre-activation (dz) and
// block partials of d loss / d log_var (ppo_net.py:29-72, ppo.py:209-217,
// 267-277): the row terms are pol_grad_row (pol_rows.hpp), shared with the
// fused head input-gradient chain's prologue
template <int NT, int AT>
__global__ void __launch_bounds__(NT)
policy_rows_grad_kernel(PolRowArgs a) {
  constexpr int AM = AT > 0 ? AT : 32;
  __shared__ PolGradShared sh;
  __shared__ float gls[NT / 64][32];
  const int A = AT > 0 ? AT : a.A;
  const int64_t N = (int64_t)a.E * a.B;
  // the thread's first row (clamped) in flight through the epoch's weights
  // and decision (the skip flag is read with the decision's scalars)
  const int64_t n0 = (int64_t)blockIdx.x * NT + threadIdx.x;
  PolGradRow<AT> x;
  x.load(a, n0 < N ? n0 : N - 1, A);
  float wsurr, wkl;
  PolGradPre pre;
  if (pol_grad_weights<8>(a, sh, wsurr, wkl, pre, a.skip)) return;
  const PolGradCols<AT> cols(pre, sh, A);
  float glv[AM];
#pragma unroll
  for (int j = 0; j < (AT > 0 ? AT : A); ++j) glv[j] = 0.f;
  const AdvNorm nadv(a, pre.mom);
  for (int64_t n = n0; n < N; n += (int64_t)gridDim.x * NT) {
    float dz[AM];
    if (n != n0) x.load(a, n, A);
    pol_grad_compute<AT>(a, cols, nadv, x, wsurr, wkl, dz, glv);
    st_row<AT>(a.dz + n * A, dz, A);
  }
  // block partials of sum_rows d/dstd (times std at the reduction: d/dlog_var)
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < (AT > 0 ? AT : A); ++j) {
    const float s = wave_sum(glv[j]);
    if (lane == 0) gls[wave][j] = s;
  }
  __syncthreads();
  for (int j = threadIdx.x; j < A; j += NT) {
    float s = 0.f;
    for (int w = 0; w < NT / 64; ++w) s += gls[w][j];
    a.lvpart[(int64_t)blockIdx.x * A + j] = s;
  }
}

__global__ void policy_decide_kernel(DecideArgs a) {
  if (threadIdx.x != 0) return;
  policy_decide_body(a, a.ps, true);
}

// single rank (no exchange between the two): the pstat reduction and the
// decision in one launch — one wave per sum, then thread 0 decides
__global__ void __launch_bounds__(kWG)
reduce_decide_kernel(const double* __restrict__ part, int nb, DecideArgs a, const int* skip) {
  if (skip && skip[0] != 0) return;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  double* out = const_cast<double*>(a.ps);
  for (int j = wave; j < PS_N; j += kNW) {
    double t = 0.0;
    for (int i = lane; i < nb; i += 64) t += part[(int64_t)i * PS_N + j];
    t = wave_sum_d(t);
    if (lane == 0) out[j] = t;
  }
  __syncthreads();
  if (threadIdx.x == 0) policy_decide_body(a, a.ps, true);
}

// value loss rows: V and the returns, both time-major [NE]; dV = 2 (V - R) / N
// and, in the last epoch, the sums of ppo.py:324-331.  A thread takes 4 rows
// per trip as float4s (V, R and dV are 16-byte aligned scratch rows), the
// NE % 4 tail one row per thread.
template <int NT>
__global__ void __launch_bounds__(NT)
value_rows_kernel(const float* __restrict__ V, const float* __restrict__ ret_tm, int B, int E,
                  float invN2, float* __restrict__ dV, double* part) {
  __shared__ double scr[NT / 64];
  double se = 0.0, d1 = 0.0, d2 = 0.0, r1 = 0.0, r2 = 0.0;
  auto acc = [&](float v, float r) {
    const float e = v - r;
    se += (double)(e * e);
    const double dd = (double)r - (double)v;
    d1 += dd; d2 += dd * dd;
    r1 += (double)r; r2 += (double)r * (double)r;
  };
  const int64_t N = (int64_t)E * B, N4 = N >> 2;
  const int64_t g0 = (int64_t)blockIdx.x * NT + threadIdx.x, gs = (int64_t)gridDim.x * NT;
  const float4* V4 = reinterpret_cast<const float4*>(V);
  const float4* R4 = reinterpret_cast<const float4*>(ret_tm);
  float4* D4 = reinterpret_cast<float4*>(dV);
  for (int64_t g = g0; g < N4; g += gs) {
    const float4 r = R4[g], v = V4[g];
    D4[g] = float4{invN2 * (v.x - r.x), invN2 * (v.y - r.y), invN2 * (v.z - r.z), invN2 * (v.w - r.w)};
    if (part) { acc(v.x, r.x); acc(v.y, r.y); acc(v.z, r.z); acc(v.w, r.w); }
  }
  for (int64_t n = 4 * N4 + g0; n < N; n += gs) {
    const float r = ret_tm[n], v = V[n];
    dV[n] = invN2 * (v - r);
    if (part) acc(v, r);
  }
  if (!part) return;
  const double sv[5] = {se, d1, d2, r1, r2};
  for (int k = 0; k < 5; ++k) {
    const double t = block_sum_d<NT>(sv[k], scr);
    if (threadIdx.x == 0) part[(int64_t)blockIdx.x * 5 + k] = t;
  }
}

// column sums of obs_iter = obs[:, :E, :] (B*E rows) in fp64 -> partials
// part[gridDim.x][2][D].  Block blk takes a contiguous run of rows; a wave
// takes every 4th row of the run with lane = column (columns past 64 in a
// second pass), four rows in flight per wave (independent accumulators,
// summed in a fixed order), then the four waves meet in LDS in wave order.
// (A column per thread striding the whole batch issued one dependent load
// per row: 31 us at C3 for a 3.6 MB read.)
__global__ void __launch_bounds__(kWG)
obs_iter_colsum_kernel(const float* __restrict__ obs, int B, int T, int E, int D,
                       double* part) {
  __shared__ double red[kWG / 64][2][64];
  const int64_t N = (int64_t)B * E;
  const int64_t per = (N + gridDim.x - 1) / gridDim.x;
  const int64_t n0 = (int64_t)blockIdx.x * per, n1 = n0 + per < N ? n0 + per : N;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int c0 = 0; c0 < D; c0 += 64) {
    const int c = c0 + lane;
    const bool ok = c < D;
    double s1[4] = {0.0, 0.0, 0.0, 0.0}, s2[4] = {0.0, 0.0, 0.0, 0.0};
    for (int64_t n = n0 + wave; n < n1; n += 16) {
      // the four rows' loads unconditional (clamped row / column) and pinned
      // before the conditional adds (same additions): under `if (ok && m < n1)`
      // each load was its own branch with a wait, four round trips per trip
      float v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int64_t m = min(n + 4 * j, n1 - 1);
        const int b = (int)(m / E), t = (int)(m - (int64_t)b * E);
        v[j] = obs[((int64_t)b * T + t) * D + min(c, D - 1)];
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) asm volatile("" : "+v"(v[j]));
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (ok && n + 4 * j < n1) {
          s1[j] += (double)v[j];
          s2[j] += (double)(v[j] * v[j]);
        }
      }
    }
    red[wave][0][lane] = (s1[0] + s1[1]) + (s1[2] + s1[3]);
    red[wave][1][lane] = (s2[0] + s2[1]) + (s2[2] + s2[3]);
    __syncthreads();
    if (wave == 0 && ok) {
      double t1 = 0.0, t2 = 0.0;
#pragma unroll
      for (int w = 0; w < kWG / 64; ++w) {
        t1 += red[w][0][lane];
        t2 += red[w][1][lane];
      }
      part[((int64_t)blockIdx.x * 2) * D + c] = t1;
      part[((int64_t)blockIdx.x * 2 + 1) * D + c] = t2;
    }
    __syncthreads();
  }
}

// torch.optim.Adam over one optimizer's parameter list [head | lstm] (two
// parameter buffers, one gradient / moment buffer), after clip_grad_norm_
// over the same list (ppo.py:243-247, 348-352).
struct AdamSplitArgs {
  float* p0; int64_t n0; float* p1; int64_t n1;
  const float* g; float* m; float* v;
  int* step; const float* lr_ptr; float beta1, beta2, eps, wd, max_norm;
  const double* part; int np;
  const int* skip; float* norm_out; int* runs;
  const int* np_dev;     // non-null: the partial count on the device (a fused sum of squares)
};
__global__ void __launch_bounds__(kWG)
adam_split_kernel(AdamSplitArgs a) {
  if (a.skip && a.skip[0] != 0) return;
  __shared__ double red[kNW];
  __shared__ float s_coef;
  const int64_t n = a.n0 + a.n1;
  // the thread's first element (every one at the launch's grid size) is loaded
  // before the norm's partials are summed: its memory latency overlaps the sum
  const int64_t i_first = (int64_t)blockIdx.x * kWG + threadIdx.x;
  float* pf = i_first < a.n0 ? a.p0 + i_first : a.p1 + (i_first - a.n0);
  float gf = 0.f, pvf = 0.f, mf = 0.f, vf = 0.f;
  if (i_first < n) {
    gf = a.g[i_first];
    pvf = *pf;
    mf = a.m[i_first];
    vf = a.v[i_first];
  }
  const int np = a.np_dev ? a.np_dev[0] : a.np;
  // every partial of the thread in flight at once: one memory round trip for
  // np <= 16 * kWG (the dW reducer's ~2300 at C3 widths; four in flight per
  // trip took three), summed in a fixed order
  constexpr int U = 16;
  double s = 0.0;
  for (int i0 = threadIdx.x; i0 < np; i0 += U * kWG) {
    double v[U];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const int i = i0 + k * kWG;
      v[k] = i < np ? a.part[i] : 0.0;
    }
#pragma unroll
    for (int k = 0; k < U; ++k) s += v[k];
  }
  s = block_sum_d(s, red);
  const int t = a.step[0];      // already bumped (sumsq_part_kernel or the dW reducer's epilogue)
  if (threadIdx.x == 0) {
    const float norm = (float)sqrt(s);
    float coef = 1.f;
    if (a.max_norm > 0.f) {
      const float cc = a.max_norm / (norm + 1e-6f);
      coef = cc < 1.f ? cc : 1.f;
    }
    s_coef = coef;
    if (blockIdx.x == 0 && a.norm_out) a.norm_out[0] = norm;
  }
  __syncthreads();
  const float coef = s_coef;
  const double bc1 = 1.0 - pow((double)a.beta1, (double)t);
  const double bc2 = 1.0 - pow((double)a.beta2, (double)t);
  const float step_size = (float)((double)a.lr_ptr[0] / bc1);
  const float bc2_sqrt = (float)sqrt(bc2);
  const float w1 = (float)(1.0 - (double)a.beta1);
  const float w2 = (float)(1.0 - (double)a.beta2);
  for (int64_t i = i_first; i < n; i += (int64_t)gridDim.x * kWG) {
    const bool fst = i == i_first;
    float* pp = fst ? pf : i < a.n0 ? a.p0 + i : a.p1 + (i - a.n0);
    float g = (fst ? gf : a.g[i]) * coef;
    float p = fst ? pvf : *pp;
    if (a.wd != 0.f) g = g + a.wd * p;
    float mi = fst ? mf : a.m[i], vi = fst ? vf : a.v[i];
    mi = mi + w1 * (g - mi);
    vi = vi * a.beta2 + (w2 * g) * g;
    const float denom = sqrtf(vi) / bc2_sqrt + a.eps;
    *pp = p + (-step_size) * (mi / denom);
    a.m[i] = mi;
    a.v[i] = vi;
  }
}

// also advances the optimizer's step counter (and the applied-epoch count):
// the Adam kernel that follows in the stream reads the bumped step
__global__ void __launch_bounds__(kWG)
sumsq_part_kernel(const float* __restrict__ g, int64_t n, double* part, const int* skip,
                  int* step, int* runs) {
  if (skip && skip[0] != 0) return;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    step[0] += 1;
    if (runs) runs[0] += 1;
  }
  __shared__ double scr[kNW];
  double s = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * kWG + threadIdx.x; i < n; i += (int64_t)gridDim.x * kWG) {
    const double v = (double)g[i];
    s += v * v;
  }
  s = block_sum_d(s, scr);
  if (threadIdx.x == 0) part[blockIdx.x] = s;
}

struct FinalArgs {
  const double* fs; int D; int64_t N; const float* lv; int A; int clip_critic;
  float* zs; float* zq; float* zc; int use_zf;
  float* stats; const int* ci; float* kl_record; int* kl_count; int kl_capacity; int Ep;
};
__global__ void rnn_final_kernel(FinalArgs a) {
  const double n = (double)a.N;
  for (int c = threadIdx.x; c < a.D && a.use_zf; c += blockDim.x) {
    a.zs[c] += (float)a.fs[FS_Z + c];                 // z_filter.py:54-56
    a.zq[c] += (float)a.fs[FS_Z + a.D + c];
  }
  if (threadIdx.x != 0) return;
  if (a.use_zf) a.zc[0] += (float)n;
  a.stats[SMI_ST_VAL_LOSS] = (float)(a.fs[FS_SE] / n);
  const double md = a.fs[FS_D] / n, mr = a.fs[FS_R] / n;
  const float vd = (float)((a.fs[FS_D2] - n * md * md) / (n - 1.0));
  const float vr = (float)((a.fs[FS_R2] - n * mr * mr) / (n - 1.0));
  a.stats[SMI_ST_VAL_EXPL_VAR] = 1.f - vd / vr;              // ppo.py:325
  float s = 0.f;
  for (int j = 0; j < a.A; ++j) s += a.lv[j];
  a.stats[SMI_ST_AVG_LOG_SIG] = s / (float)a.A;             // ppo.py:571
  a.stats[SMI_ST_EPOCHS_RUN] = (float)a.ci[CI_RUNS];
  if (a.Ep > 0) {                                            // ppo.py:559
    const int k = a.kl_count[0];
    if (k < a.kl_capacity) a.kl_record[k] = a.stats[SMI_ST_POL_KL];
    a.kl_count[0] = k + 1;
  }
}

// ------------------------------------------------------------ host phases

// workgroups of the statistics pass: at most one resident round (its register
// count leaves 3 one-wave blocks per SIMD, so the 4096-block cap of rnn_nblk
// ran a second, partly filled round: 0.34 of HBM at 65536 segments)
// adapt mode, 8 actions: the statistics pass with its per-column terms in
// LDS and one row in flight per thread (168 -> 118 VGPRs: four waves per SIMD
// instead of three, to cover the rows' cold HBM reads)
template <int NT>
__global__ void __launch_bounds__(NT)
policy_rows_stats_lean_kernel(PolRowArgs a) {
  if (a.skip && a.skip[0] != 0) return;
  constexpr int AT = 8;
  __shared__ PolStatsColsLds sc;
  __shared__ double scr[NT / 64][PS_N];
  pol_stats_cols_fill(sc, a.lv, a.ref_lv, AT);
  __syncthreads();
  double acc[PS_N];
#pragma unroll
  for (int k = 0; k < PS_N; ++k) acc[k] = 0.0;
  const int64_t N = (int64_t)a.E * a.B;
  const AdvNorm nadv(a);
  for (int64_t n = (int64_t)blockIdx.x * NT + threadIdx.x; n < N; n += (int64_t)gridDim.x * NT) {
    float m[AT], rm[AT], ac[AT];
    ld_row<AT>(m, a.mu + n * AT, AT);
    ld_row<AT>(rm, a.refmu + n * AT, AT);
    ld_fields<AT>(ac, a.rowin, N, n, 0, AT);
    const float adv = a.rowin[rin_idx(row_w(AT), n, rin_adv(AT))];
    const float bl = a.rowin[rin_idx(row_w(AT), n, rin_bl(AT))];
    const float rbd = a.rowin[rin_idx(row_w(AT), n, rin_rbd(AT))];
    pol_stats_row_adapt<AT>(a, sc, nadv, m, rm, ac, bl, rbd, adv, a.ret_tm[n], acc);
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < PS_N; ++k) {
    const double v = wave_sum_d(acc[k]);
    if (lane == 0) scr[wave][k] = v;
  }
  __syncthreads();
  if (threadIdx.x < PS_N) {
    double t = 0.0;
#pragma unroll
    for (int w = 0; w < NT / 64; ++w) t += scr[w][threadIdx.x];
    a.part[(int64_t)blockIdx.x * PS_N + threadIdx.x] = t;
  }
}

// off unless SMI_STATS_LEAN=1: at 65536 segments 0.381 vs 0.377 of HBM (the
// pass reads its rows cold either way)
static bool use_stats_lean() {
  static const bool on = [] { const char* e = getenv("SMI_STATS_LEAN"); return e && e[0] == '1'; }();
  return on;
}

template <bool FUSE>
static int pol_stats_blocks(int A, int64_t rows) {
  static int cap[2][9] = {};
  const int ai = A >= 1 && A <= 8 ? A : 0;
  int& c = cap[FUSE][ai];
  if (!c) {
    if (!FUSE && ai == 8 && use_stats_lean()) c = resident_grid(policy_rows_stats_lean_kernel<kRowNT>, kRowNT, 0);
    else switch (ai) {
      case 1: c = resident_grid(policy_rows_stats_kernel<kRowNT, 1, FUSE>, kRowNT, 0); break;
      case 2: c = resident_grid(policy_rows_stats_kernel<kRowNT, 2, FUSE>, kRowNT, 0); break;
      case 3: c = resident_grid(policy_rows_stats_kernel<kRowNT, 3, FUSE>, kRowNT, 0); break;
      case 4: c = resident_grid(policy_rows_stats_kernel<kRowNT, 4, FUSE>, kRowNT, 0); break;
      case 5: c = resident_grid(policy_rows_stats_kernel<kRowNT, 5, FUSE>, kRowNT, 0); break;
      case 6: c = resident_grid(policy_rows_stats_kernel<kRowNT, 6, FUSE>, kRowNT, 0); break;
      case 7: c = resident_grid(policy_rows_stats_kernel<kRowNT, 7, FUSE>, kRowNT, 0); break;
      case 8: c = resident_grid(policy_rows_stats_kernel<kRowNT, 8, FUSE>, kRowNT, 0); break;
      default: c = resident_grid(policy_rows_stats_kernel<kRowNT, 0, FUSE>, kRowNT, 0); break;
    }
    if (c < 1) c = 1;
  }
  const int nb = rnn_nblk(rows, kRowNT);
  return nb < c ? nb : c;
}

template <bool FUSE>
static void launch_pol_stats(int A, int nb, const PolRowArgs& p, hipStream_t st) {
  if (!FUSE && A == 8 && use_stats_lean()) {
    hipLaunchKernelGGL((policy_rows_stats_lean_kernel<kRowNT>), dim3(nb), dim3(kRowNT), 0, st, p);
    return;
  }
  switch (A) {   // compile-time action widths 1..8 (registers); others generic
    case 1: hipLaunchKernelGGL((policy_rows_stats_kernel<kRowNT, 1, FUSE>), dim3(nb), dim3(kRowNT), 0, st, p); break;
    case 2: hipLaunchKernelGGL((policy_rows_stats_kernel<kRowNT, 2, FUSE>), dim3(nb), dim3(kRowNT), 0, st, p); break;
    case 3: hipLaunchKernelGGL((policy_rows_stats_kernel<kRowNT, 3, FUSE>), dim3(nb), dim3(kRowNT), 0, st, p); break;
    case 4: hipLaunchKernelGGL((policy_rows_stats_kernel<kRowNT, 4, FUSE>), dim3(nb), dim3(kRowNT), 0, st, p); break;
    case 5: hipLaunchKernelGGL((policy_rows_stats_kernel<kRowNT, 5, FUSE>), dim3(nb), dim3(kRowNT), 0, st, p); break;
    case 6: hipLaunchKernelGGL((policy_rows_stats_kernel<kRowNT, 6, FUSE>), dim3(nb), dim3(kRowNT), 0, st, p); break;
    case 7: hipLaunchKernelGGL((policy_rows_stats_kernel<kRowNT, 7, FUSE>), dim3(nb), dim3(kRowNT), 0, st, p); break;
    case 8: hipLaunchKernelGGL((policy_rows_stats_kernel<kRowNT, 8, FUSE>), dim3(nb), dim3(kRowNT), 0, st, p); break;
    default: hipLaunchKernelGGL((policy_rows_stats_kernel<kRowNT, 0, FUSE>), dim3(nb), dim3(kRowNT), 0, st, p); break;
  }
}

static int grid_of(int64_t n, int cap = 1024) {
  int64_t g = (n + kWG - 1) / kWG;
  if (g < 1) g = 1;
  return (int)(g < cap ? g : cap);
}

#define RC(x) do { const int rc_ = (x); if (rc_) return rc_; } while (0)

// zf_tmajor_kernel: kZfRows (x rows per load) rows per wave and trip, 4 waves
// per block, at most 2048 blocks
static int zf_grid(int64_t rows) {
  int64_t g = (rows + 4 * kZfRows - 1) / (4 * kZfRows);
  if (g < 1) g = 1;
  return (int)(g < 2048 ? g : 2048);
}

// the time-major z-filtered copy of the batch's low-dim observations: the tile
// transpose where its shape conditions hold, else the row-per-wave kernel.
// form: 0 = that choice, 1 = the row kernel, 2 = the float2 tile, 3 = the
// float4 tile, 4 = the pipelined float4 tile writing whole padded rows (zeros
// in columns D..ldo-1; the learner's choice only with pad_ok: nothing else
// writes there), 5 = the one-shot float4 tile writing whole padded rows
// (smi_zfilter_tmajor's test / bench selection; a form whose shape conditions
// fail is SMI_E_ARG)
static int launch_zf_tmajor(const float* obs, const float* obs_next, int B, int T, int S, int D,
                            int use_zf, const float* zs, const float* zq, const float* zc,
                            float eps, float* out, int ldo, hipStream_t st, int form = 0,
                            bool pad_ok = false) {
  if (D <= 0 || S <= 0) return SMI_OK;
  auto a8 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 7) == 0; };
  auto a16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  const size_t tl = ((size_t)2 * round4(D) + (size_t)kZfSeg * S * D) * 4;
  const size_t tl4 = ((size_t)2 * round4(D) + round4(kZfSeg * T * D) + (size_t)kZfSeg * D) * 4;
  const bool tile_ok = D % 2 == 0 && D <= 128 && ldo % 2 == 0 && a8(obs) && a8(obs_next) &&
                       a8(out) && D / 2 * kZfSeg <= kWG && tl <= 64 * 1024;
  const bool tile4_ok = ldo % 4 == 0 && a16(obs) && a16(obs_next) && a16(out) && tl4 <= 64 * 1024;
  const bool pad4_ok = tile4_ok && ldo == round4(D) && kZfSeg * (ldo / 4) <= kWG;
  const size_t tlp = ((size_t)2 * round4(D) +
                      2 * ((size_t)round4(kZfSeg * T * D) + round4(kZfSeg * D))) * 4;
  const bool pipe_ok = pad4_ok && kZfSeg * T * D <= 4 * kZfNR * kWG && kZfSeg * D <= 4 * kWG &&
                       tlp <= 150 * 1024;
  // SMI_ZF_PIPE=0: the one-shot padded-row tile (A/B)
  static const bool pipe_on = [] { const char* e = getenv("SMI_ZF_PIPE"); return !(e && e[0] == '0'); }();
  static const bool tile_on = [] { const char* e = getenv("SMI_ZF_TILE"); return !(e && e[0] == '0'); }();
  static const bool force = [] { const char* e = getenv("SMI_ZF_TILE_FORCE"); return e && e[0] == '1'; }();
  // SMI_ZF_TILE4=0: the float2 tile (A/B)
  static const bool t4_on = [] { const char* e = getenv("SMI_ZF_TILE4"); return !(e && e[0] == '0'); }();
  if (form == 0) {
    // (from 4096 segments: at C3's 1024 the 128 tile workgroups took 14.5 us
    // against 9.7 for the row kernel; at 65536, 146 against 169 us)
    form = 1;
    if (tile_on && (B >= 4096 || force)) {
      if (t4_on && pad_ok && pipe_on && pipe_ok) form = 4;
      else if (t4_on && pad_ok && pad4_ok) form = 5;
      else if (tile_ok) form = 2;
      else if (tile4_ok) form = 3;
    }
  }
  const int nb = (B + kZfSeg - 1) / kZfSeg;
  if (form == 4) {
    if (!pipe_ok) return set_error(SMI_E_ARG, "zf_tmajor: pipelined padded rows do not fit");
    allow_lds(zf_pipe_kernel, tlp);
    static int cap = 0;
    if (!cap) cap = std::max(1, resident_grid(zf_pipe_kernel, kWG, tlp));
    hipLaunchKernelGGL(zf_pipe_kernel, dim3(std::min(nb, cap)), dim3(kWG), tlp, st, obs, obs_next,
                       B, T, S, D, use_zf, zs, zq, zc, eps, out, ldo);
    return check_launch("zf_pipe_kernel");
  }
  if (form == 3 || form == 5) {
    if (!tile4_ok) return set_error(SMI_E_ARG, "zf_tmajor: float4 tile needs 16-byte alignment");
    if (form == 5 && !pad4_ok) return set_error(SMI_E_ARG, "zf_tmajor: padded rows need ldo == round4(D)");
    allow_lds(zf_tile4_kernel, tl4);
    hipLaunchKernelGGL(zf_tile4_kernel, dim3(nb), dim3(kWG), tl4, st, obs, obs_next, B, T, S, D,
                       use_zf, zs, zq, zc, eps, out, ldo, form == 5 ? 1 : 0);
    return check_launch("zf_tile4_kernel");
  }
  if (form == 2) {
    if (!tile_ok) return set_error(SMI_E_ARG, "zf_tmajor: float2 tile needs even D, 8-byte alignment");
    allow_lds(zf_tile_kernel, tl);
    hipLaunchKernelGGL(zf_tile_kernel, dim3(nb), dim3(kWG), tl, st, obs, obs_next, B, T, S, D,
                       use_zf, zs, zq, zc, eps, out, ldo);
    return check_launch("zf_tile_kernel");
  }
  if (D > 128) return set_error(SMI_E_ARG, "zf_tmajor: D > 128");
  const size_t zlds = (size_t)2 * round4(D) * 4;
  hipLaunchKernelGGL(zf_tmajor_kernel, dim3(zf_grid((int64_t)S * B)), dim3(kWG), zlds, st, obs,
                     obs_next, B, T, S, D, use_zf, zs, zq, zc, eps, out, ldo);
  return check_launch("zf_tmajor_kernel");
}

int launch_zfilter_tmajor(const float* obs, const float* obs_next, int B, int T, int S, int D,
                          int use_zf, const float* zs, const float* zq, const float* zc, float eps,
                          float* out, int ldo, int form, hipStream_t st) {
  return launch_zf_tmajor(obs, obs_next, B, T, S, D, use_zf, zs, zq, zc, eps, out, ldo, st, form,
                          form >= 4);
}

struct Head {   // one MLP head over rows of an activation matrix
  const float* P; MlpLayout L; int in, h1, h2, out, tanh_out;
};

bool head_fused_ok(int in, int64_t ldx, int h1, int h2, int out, const float* X,
                   const float* W1, const float* W2, const float* W3);
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

static bool head_fused(const Head& h, const float* X, int64_t ldx) {
  return head_fused_ok(h.in, ldx, h.h1, h.h2, h.out, X, h.P + h.L.fW1, h.P + h.L.fW2,
                       h.P + h.L.fW3);
}

// forward: X[rows][ldx] -> HA1 -> HA2 -> Y ([rows][out]); one fused launch
// (head_kernels.hip) when the shapes allow, which with wT also writes W1^T | W2^T
// for a fused backward of the same parameters
// vret / vgrad / vscale: the value-loss gradient written by the fused forward
// (out == 1); *vdone tells whether it was (the layer-GEMM path does not)
// ps: the policy statistics epilogue (the fused path only: head_fwd_ps_ok)
static int head_fwd(const Head& h, const float* X, int64_t ldx, int64_t rows, float* HA1,
                    float* HA2, float* Y, hipStream_t st, const int* skip, float* wT = nullptr,
                    const float* vret = nullptr, float* vgrad = nullptr, float vscale = 0.f,
                    bool* vdone = nullptr, const PolRowArgs* ps = nullptr,
                    double* vpart = nullptr, bool keep_act = true) {
  const MlpLayout& L = h.L;
  if (vdone) *vdone = false;
  if (head_fused(h, X, ldx)) {
    // keep_act false: no backward follows (the GAE critic pass, PREP's
    // reference forward, the KL check after the last policy update), so the
    // fused chain skips the HA1 / HA2 copy-outs (the layer-GEMM path below
    // needs them as its intermediates)
    if (!keep_act) HA1 = HA2 = nullptr;
    const bool ve = vgrad && h.out == 1;
    if (vdone) *vdone = ve;
    return launch_head_fwd_fused(X, ldx, rows, h.in, h.P + L.fW1, h.P + L.fb1, h.h1, h.P + L.fW2,
                                 h.P + L.fb2, h.h2, h.P + L.fW3, h.P + L.fb3, h.out, h.tanh_out,
                                 HA1, HA2, Y, h.out, wT, wT ? wT + (int64_t)h.in * h.h1 : nullptr,
                                 st, skip, ve ? vret : nullptr, ve ? vgrad : nullptr, vscale, ps,
                                 ve ? vpart : nullptr);
  }
  if (ps) return set_error(SMI_E_ARG, "head_forward: the statistics epilogue needs the fused head");
  const int M = (int)rows;
  RC(launch_linear_fwd(X, ldx, M, h.in, h.P + h.L.fW1, h.in, h.P + h.L.fb1, h.h1, ACT_RELU, HA1,
                       h.h1, st, skip));
  RC(launch_linear_fwd(HA1, h.h1, M, h.h1, h.P + h.L.fW2, h.h1, h.P + h.L.fb2, h.h2, ACT_RELU, HA2,
                       h.h2, st, skip));
  return launch_linear_fwd(HA2, h.h2, M, h.h2, h.P + h.L.fW3, h.h2, h.P + h.L.fb3, h.out,
                           h.tanh_out ? ACT_TANH : ACT_NONE, Y, h.out, st, skip);
}

// backward from dZ (gradient at the last layer's pre-activation) into the flat
// gradient image G (same layout as P); input-gradient columns [dx0, dx0+dxn)
// to dXout ([rows][dxn], masked by dxmask > 0 when given; dxn == 0: none).
// Inside a dW group (stem_backward) the weight gradients are queued and run
// as one grouped launch at the flush.
// pg: the policy-gradient prologue (dZ computed from the policy rows by the
// fused chain itself); only on the fused path (head_bwd_pg_ok)
static int head_bwd(const Head& h, const float* dZ, const float* X, int64_t ldx, int64_t rows,
                    const float* HA1, const float* HA2, float* dH1, float* dH2, float* G,
                    int dx0, int dxn, const float* dxmask, int64_t ldm, float* dXout,
                    hipStream_t st, const int* skip, const float* wT = nullptr,
                    const PolRowArgs* pg = nullptr) {
  const int M = (int)rows;
  const MlpLayout& L = h.L;
  if (wT && dxn <= 320 && head_fused(h, X, ldx)) {
    // the input-gradient chain in one launch (dH2, dH1, dX), then the three
    // weight gradients (queued into the phase's dW group when one is open)
    RC(launch_head_bwd_fused(dZ, h.out, rows, h.P + L.fW3, wT + (int64_t)h.in * h.h1, wT, h.h1,
                             h.h2, dx0, dxn, HA1, HA2, dH2, dH1, dXout, dxn, dxmask, ldm, st,
                             skip, pg));
    RC(launch_linear_bwd_dw(dZ, h.out, M, h.out, HA2, h.h2, h.h2, G + L.fW3, h.h2, G + L.fb3, 0,
                            st, skip));
    RC(launch_linear_bwd_dw(dH2, h.h2, M, h.h2, HA1, h.h1, h.h1, G + L.fW2, h.h1, G + L.fb2, 0,
                            st, skip));
    return launch_linear_bwd_dw(dH1, h.h1, M, h.h1, X, ldx, h.in, G + L.fW1, h.in, G + L.fb1, 0,
                                st, skip);
  }
  if (pg) return set_error(SMI_E_ARG, "head_backward: the policy prologue needs the fused chain");
  RC(launch_linear_bwd_dw(dZ, h.out, M, h.out, HA2, h.h2, h.h2, G + L.fW3, h.h2, G + L.fb3, 0, st,
                          skip));
  RC(launch_linear_bwd_dx(dZ, h.out, M, h.out, h.P + L.fW3, h.h2, h.h2, HA2, h.h2, dH2, h.h2, st,
                          skip));
  RC(launch_linear_bwd_dw(dH2, h.h2, M, h.h2, HA1, h.h1, h.h1, G + L.fW2, h.h1, G + L.fb2, 0, st,
                          skip));
  RC(launch_linear_bwd_dx(dH2, h.h2, M, h.h2, h.P + L.fW2, h.h1, h.h1, HA1, h.h1, dH1, h.h1, st,
                          skip));
  RC(launch_linear_bwd_dw(dH1, h.h1, M, h.h1, X, ldx, h.in, G + L.fW1, h.in, G + L.fb1, 0, st,
                          skip));
  if (dxn <= 0) return SMI_OK;
  return launch_linear_bwd_dx(dH1, h.h1, M, h.h1, h.P + L.fW1 + dx0, h.in, dxn, dxmask, ldm, dXout,
                              dxn, st, skip);
}

// per-layer regions of the LSTM buffers
static float* hbuf_of(const RnnDims& d, const RnnScratch& s, int l) {
  return s.hbuf + (int64_t)l * (d.S1 + 1) * d.B * d.H;
}
static float* cbuf_of(const RnnDims& d, const RnnScratch& s, int l) {
  return s.cbuf + (int64_t)l * (d.E + 1) * d.B * d.H;
}
static float* gates_of(const RnnDims& d, const RnnScratch& s, int l) {
  return s.gates + (int64_t)l * d.NE * d.G4;
}
static float* dgates_of(const RnnDims& d, const RnnScratch& s, int l) {
  return s.dgates + (int64_t)l * d.NE * d.G4;
}

struct LstmP { const float *Wih, *Whh, *bih, *bhh; };
static LstmP lstm_params(const float* p, int D, int H) {
  LstmP l;
  l.Wih = p;
  l.Whh = p + (int64_t)4 * H * D;
  l.bih = l.Whh + (int64_t)4 * H * H;
  l.bhh = l.bih + 4 * H;
  return l;
}
// layer l of a stem buffer [layer 0 (in Din) | layer 1 (in H) | ...]
static LstmP lstm_layer(const RnnDims& d, const float* p, int l) {
  return l == 0 ? lstm_params(p, d.Din, d.H)
                : lstm_params(p + d.nL0 + (int64_t)(l - 1) * d.nLk, d.H, d.H);
}

// the stacked LSTM over S steps from (h0, c0) ([L][B][H] each): layer 0 reads X
// (fused input projection when it fits, else xproj GEMM + recurrence), layer
// l >= 1 reads layer l-1's outputs hbuf_l-1[1..S]; keep: store the cell states
// and gate activations of every layer for a backward
// keep_steps: with keep, the cell states / gates are stored for the first
// keep_steps steps only (0: all S; the GAE pass over S1 steps keeps E)
static int lstm_forward(const RnnDims& d, const float* P, const float* X, int S, const float* h0,
                        const float* c0, const RnnScratch& s, bool keep, hipStream_t st,
                        const int* skip, int keep_steps = 0) {
  const int64_t BH = (int64_t)d.B * d.H;
  for (int l = 0; l < d.L; ++l) {
    const LstmP lp = lstm_layer(d, P, l);
    const float* Xl = l == 0 ? X : hbuf_of(d, s, l - 1) + BH;
    const int64_t ldx = l == 0 ? d.ldx : d.H;
    const int din = l == 0 ? d.Din : d.H;
    float* hb = hbuf_of(d, s, l);
    float* cb = keep ? cbuf_of(d, s, l) : nullptr;
    float* gt = keep ? gates_of(d, s, l) : nullptr;
    const int rf = launch_lstm_fwd_x(Xl, ldx, din, lp.Wih, lp.bih, lp.Whh, lp.bhh, h0 + l * BH,
                                     c0 + l * BH, S, d.B, d.H, hb, cb, gt, st, skip, keep_steps);
    if (rf == SMI_E_NOFIT) {
      const int64_t rows = (int64_t)S * d.B;
      RC(launch_linear_fwd(Xl, ldx, (int)rows, din, lp.Wih, din, lp.bih, d.G4, ACT_NONE, s.xproj,
                           d.G4, st, skip));
      RC(launch_lstm_fwd(s.xproj, lp.Whh, lp.bhh, h0 + l * BH, c0 + l * BH, S, d.B, d.H, hb, cb, gt,
                         st, skip, keep_steps));
    } else if (rf) {
      return rf;
    }
  }
  return SMI_OK;
}

// gradients of the stacked LSTM's parameters (flat layout) from dh [E][B][H] at
// the top layer's outputs: BPTT layer by layer downwards, each layer's input
// gradient dgates_l W_ih_l (no activation between layers) the dh of the layer
// below; the weight gradients over [x_t | h_{t-1}] join the phase's dW group
static int lstm_backward(const RnnDims& d, const float* P, float* G, const RnnScratch& s,
                         hipStream_t st, const int* skip) {
  const int64_t BH = (int64_t)d.B * d.H;
  const int M = (int)d.NE;
  static const int fused = [] { const char* e = getenv("SMI_LSTM_DW2"); return e ? atoi(e) : 1; }();
  for (int l = d.L - 1; l >= 0; --l) {
    const LstmP lp = lstm_layer(d, P, l);
    float* dg = dgates_of(d, s, l);
    float* hb = hbuf_of(d, s, l);
    // one layer, no pixel stem: the BPTT shares its launch with the heads'
    // weight gradients queued so far (their partials stay reserved in the
    // workspace until the group's flush: workspace_reserve; one layer, so the
    // pre entries (<= 6 after tail splits) and this layer's (<= 2) fit the
    // reducer's 8)
    int rb = SMI_E_NOFIT;
    if (d.L == 1 && d.F == 0)
      rb = launch_lstm_bwd_dw(s.dh, gates_of(d, s, l), cbuf_of(d, s, l), lp.Whh, d.E, d.B, d.H, dg,
                              st, skip);
    if (rb == SMI_E_NOFIT)
      RC(launch_lstm_bwd(s.dh, gates_of(d, s, l), cbuf_of(d, s, l), lp.Whh, d.E, d.B, d.H, dg, st,
                         skip));
    else if (rb)
      return rb;
    const int din = l == 0 ? d.Din : d.H;
    const float* Xl = l == 0 ? s.Xz : hbuf_of(d, s, l - 1) + BH;
    const int64_t ldx = l == 0 ? d.ldx : d.H;
    float* gWih = G + (l == 0 ? 0 : d.nL0 + (int64_t)(l - 1) * d.nLk);
    float* gWhh = gWih + (int64_t)4 * d.H * din;
    float* gbih = gWhh + (int64_t)4 * d.H * d.H;
    float* gbhh = gbih + d.G4;
    if (!fused) {     // A/B: the two launches over the layer input and hbuf
      RC(launch_linear_bwd_dw(dg, d.G4, M, d.G4, Xl, ldx, din, gWih, din, gbih, 0, st, skip));
      RC(launch_linear_bwd_dw(dg, d.G4, M, d.G4, hb, d.H, d.H, gWhh, d.H, gbhh, 0, st, skip));
    } else {
      // W_ih over x_t, W_hh over h_{t-1} (hbuf[0..E-1], hbuf[0] = h0) and the
      // shared bias gradient in ONE launch over [x_t | h_{t-1}]
      RC(launch_linear_bwd_dw2(dg, d.G4, M, d.G4, Xl, ldx, din, hb, d.H, d.H, gWih, din, gWhh,
                               d.H, gbih, gbhh, st, skip));
    }
    if (l > 0)        // dh of layer l-1's outputs (steps 1..E) = dgates_l W_ih_l
      RC(launch_linear_bwd_dx(dg, d.G4, M, d.G4, lp.Wih, d.H, d.H, nullptr, 0, s.dh, d.H, st, skip));
  }
  return SMI_OK;
}

static PixRows pix_rows(const smi_ppo_rnn_args& a, const RnnDims& d) {
  return PixRows{a.pixels, a.pixels_next, d.B, d.T, d.G.img};
}

// CNN features of the first S time steps into X[:, D:] (ldx = Din); A1 kept
// for a backward when non-null
static int cnn_features(const smi_ppo_rnn_args& a, const RnnDims& d, const float* cnn, int S,
                        float* X, float* A1, const RnnScratch& s, hipStream_t st,
                        const int* skip) {
  if (d.F == 0) return SMI_OK;
  return cnn_forward(cnn, pix_rows(a, d), d.G.C, d.G.H, d.G.W, d.F, (int64_t)S * d.B, A1, s.A2,
                     X + d.D, d.ldx, st, skip);
}

// CNN backward from dF = dL/d(features) * relu'(features) in s.dF
static int cnn_bwd_from_dF(const smi_ppo_rnn_args& a, const RnnDims& d, const float* cnn,
                           float* Gc, const RnnScratch& s, hipStream_t st, const int* skip) {
  return cnn_backward(cnn, pix_rows(a, d), d.G.C, d.G.H, d.G.W, d.F, d.NE, s.A1, s.A2, s.dF, d.F,
                      Gc, s.dA2, s.cpart, st, skip);
}

// pixel-stem gradient (into Gc) from the LSTM gate gradients of the E steps:
// dF = relu'(F) * (dgates W_ih[:, D:]), then the CNN backward
static int cnn_grad(const smi_ppo_rnn_args& a, const RnnDims& d, const LstmP& l, const float* cnn,
                    float* Gc, const RnnScratch& s, hipStream_t st, const int* skip) {
  if (d.F == 0) return SMI_OK;
  RC(launch_linear_bwd_dx(dgates_of(d, s, 0), d.G4, (int)d.NE, d.G4, l.Wih + d.D, d.Din, d.F,
                          s.Xz + d.D, d.ldx, s.dF, d.F, st, skip));
  return cnn_bwd_from_dF(a, d, cnn, Gc, s, st, skip);
}

// the policy / value features the heads read: LSTM outputs hbuf[1..] ([S][B][H])
// or, without the LSTM (MLP policy), the stem input itself ([S][B][Din])
static const float* head_in(const RnnDims& d, const RnnScratch& s, const float* X) {
  return d.H > 0 ? hbuf_of(d, s, d.L - 1) + (int64_t)d.B * d.H : X;
}

// backward of one head into G (+ the stem below it): LSTM BPTT and/or CNN
static int stem_backward_chain(const smi_ppo_rnn_args& a, const RnnDims& d, const Head& hd,
                               const LstmP& lm, const float* cnn, float* G, const RnnScratch& s,
                               int64_t n_head, hipStream_t st, const int* skip,
                               const PolRowArgs* pg) {
  const float* X = head_in(d, s, s.Xz);
  if (d.H > 0) {
    RC(head_bwd(hd, s.dOUT, X, d.Hld, d.NE, s.HA1, s.HA2, s.dH1, s.dH2, G, 0, d.H, nullptr, 0,
                s.dh, st, skip, s.wT, pg));
    RC(lstm_backward(d, a.lstm, G + n_head, s, st, skip));
    return cnn_grad(a, d, lm, cnn, G + n_head + d.nL, s, st, skip);
  }
  if (pg) return set_error(SMI_E_ARG, "ppo_rnn: the policy prologue needs the LSTM stem");
  // MLP policy: the first head layer's input gradient over the CNN columns only
  RC(head_bwd(hd, s.dOUT, X, d.Hld, d.NE, s.HA1, s.HA2, s.dH1, s.dH2, G, d.D, d.F, s.Xz + d.D,
              d.ldx, s.dF, st, skip, s.wT));
  if (d.F == 0) return SMI_OK;
  return cnn_bwd_from_dF(a, d, cnn, G + n_head, s, st, skip);
}

// every weight gradient of the phase (head layers + LSTM) queued and run as
// one grouped launch after the input-gradient chain and BPTT
// ex: the reducer's epilogue task (the log_var gradient, the clip-norm partials)
static int stem_backward(const smi_ppo_rnn_args& a, const RnnDims& d, const Head& hd,
                         const LstmP& lm, const float* cnn, float* G, const RnnScratch& s,
                         int64_t n_head, hipStream_t st, const int* skip,
                         const DwEpilogue* ex = nullptr, const PolRowArgs* pg = nullptr) {
  dw_group_begin();
  if (ex) RC(dw_group_epilogue(*ex));
  const int rc = stem_backward_chain(a, d, hd, lm, cnn, G, s, n_head, st, skip, pg);
  const int rf = dw_group_flush(st);     // always flush: nothing stays queued after an error
  return rc ? rc : rf;
}

static float c_loglik_of(int A) { return (float)(0.5 * log(2.0 * 3.141592653589793) * (double)A); }
static float c_entropy_of(int A) {
  return (float)(0.5 * log(2.0 * 3.141592653589793 * 2.718281828459045) * (double)A);
}

int64_t ppo_rnn_scratch_bytes(int B, int T, int Hz, int D, int H, int L, int h1, int h2, int A, int c1,
                              int c2, int pc, int ph, int pw, int F) {
  return 4 * rnn_scratch(rnn_dims(B, T, Hz, D, H, h1, h2, A, c1, c2, pc, ph, pw, F, L), nullptr)
                 .total_floats;
}

static PolRowArgs pol_rows(const smi_ppo_rnn_args& a, const RnnDims& d, const RnnScratch& s) {
  PolRowArgs p{};
  p.B = d.B; p.T = d.T; p.E = d.E; p.A = d.A; p.mode = a.mode;
  p.mu = s.OUT; p.lv = a.actor + d.LA.flv; p.refmu = s.refmu; p.ref_lv = a.ref_actor + d.LA.flv;
  p.actions = a.actions; p.behave = a.behave; p.adv = s.adv; p.ret = s.ret;
  p.rowin = s.rowin; p.ret_tm = s.ret_tm;
  p.moments = a.moments; p.norm_adv = a.norm_adv; p.c_ll = c_loglik_of(d.A);
  p.hyper = a.hyper; p.skip = s.ci + CI_STOP;
  p.part = s.part; p.dz = s.dOUT; p.lvpart = s.lvpart; p.cf = s.cf;
  return p;
}

// One rank with no pixel stem: the optimizer's clip_grad_norm_ partials come
// from the dW group's reducer (every gradient of [head | lstm] but log_var is a
// reducer output, log_var is the reducer's epilogue task), so the APPLY phases
// run Adam alone.  Data parallel: the norm is of the all-reduced gradient, so
// the sums of squares stay in APPLY (sumsq_part_kernel); with the pixel stem
// the CNN gradient is not a reducer output.
// Every weight gradient of both optimizers must join the group for that
// (dw_group_takes: heads wider than 511 or 4H > 512 run outside it); the flush
// also fails loudly if one ran outside an open bracket with the fused norm.
static bool fused_clip_norm(const smi_ppo_rnn_args& a, const RnnDims& d) {
  static const bool off = [] { const char* e = getenv("SMI_FUSED_NORM"); return e && e[0] == '0'; }();
  if (off || a.B_global != a.B || d.F != 0 || d.L > 3 || fault() != 0) return false;
  const bool heads = dw_group_takes(d.h1, d.Hin + 1) && dw_group_takes(d.h2, d.h1 + 1) &&
                     dw_group_takes(d.A, d.h2 + 1) && dw_group_takes(d.c1, d.Hin + 1) &&
                     dw_group_takes(d.c2, d.c1 + 1) && dw_group_takes(1, d.c2 + 1);
  const bool stem = d.H == 0 || (dw_group_takes(d.G4, d.ldx + d.H + 1) &&
                                 (d.L == 1 || dw_group_takes(d.G4, d.H + d.H + 1)));
  return heads && stem;
}

// the GAE critic pass (T + 1 steps) and PREP's reference-policy forward (E
// steps) as ONE recurrence launch (two weight sets over two inputs, B
// workgroups each): one LSTM layer, no pixel stem, the one-segment form for 2B
// segments, PREP issued after GAE on the same stream (a.prep_independent == 0:
// the caller's explicit statement, no environment read here); GAE then also
// forms PREP's z-filtered input and PREP runs the reference head only.
// SMI_GAE_DUAL=0: two launches (A/B knob)
static bool gae_prep_dual(const smi_ppo_rnn_args& a, const RnnDims& d) {
  static const bool off = [] { const char* e = getenv("SMI_GAE_DUAL"); return e && e[0] == '0'; }();
  return !off && a.prep_independent == 0 && d.H > 0 && d.L == 1 && d.F == 0 &&
         lstm_fwd_x_dual_fits(d.B, d.B, d.S1 > d.E ? d.S1 : d.E, d.H, d.Din);
}

// adapt mode with the LSTM stem, 8 actions and the fused head chain at a
// rank's batch (< 16384 rows: one row tile per workgroup): the policy-gradient
// row pass runs as that chain's prologue (head_kernels.hip, pol_rows.hpp;
// SMI_POL_HEAD=0: its own launch, 1: at any batch; A/B knob); one log_var
// partial per chain workgroup (<= the 4096 of s.lvpart).  Measured: 128
// segments 2.947 -> 2.929 ms per learn; 1024 segments 6.98 -> 7.05 ms (the
// 32-row workgroups' serial prologue costs more than the launch it saves)
static bool pol_head_grad(const smi_ppo_rnn_args& a, const RnnDims& d, const RnnScratch& s,
                          const Head& actor) {
  static const int knob = [] { const char* e = getenv("SMI_POL_HEAD"); return e && e[0] ? atoi(e) : -1; }();
  if (knob == 0) return false;
  return a.mode != 0 && d.H > 0 && d.A == 8 && d.H <= 320 && (knob == 1 || d.NE < 16384) &&
         head_fused(actor, head_in(d, s, s.Xz), d.Hld) && head_bwd_blocks(d.NE) <= 4096;
}

// adapt mode, 8 actions, 300 x 200-class heads on the fused path: the policy
// statistics row pass as the head forward's epilogue (one launch fewer per
// policy epoch); one PS_N partial per head workgroup (<= 4096 of them).  Off
// unless SMI_POL_STATS_HEAD=1 (A/B knob): measured 2.933 vs 2.928 ms at 128
// segments, 6.986 vs 6.999 ms at C3 — the workgroups' serial row epilogue
// (+6 / +10 us per forward) costs what the launch it removes did
static bool pol_head_stats(const smi_ppo_rnn_args& a, const RnnDims& d, const RnnScratch& s,
                           const Head& actor) {
  static const bool on = [] { const char* e = getenv("SMI_POL_STATS_HEAD"); return e && e[0] == '1'; }();
  return on && a.mode != 0 && d.A == 8 && head_fwd_ps_ok(d.h1, d.h2, d.A) &&
         head_fused(actor, head_in(d, s, s.Xz), d.Hld) && head_bwd_blocks(d.NE) <= 4096;
}
// the partials the policy statistics pass wrote (its grid, or the head's)
static int pol_stats_nb(const smi_ppo_rnn_args& a, const RnnDims& d, const RnnScratch& s,
                        const Head& actor) {
  if (a.mode == 0) return pol_stats_blocks<true>(d.A, d.NE);
  return pol_head_stats(a, d, s, actor) ? head_bwd_blocks(d.NE) : pol_stats_blocks<false>(d.A, d.NE);
}

// adapt mode, one rank, a policy epoch that trains: the decision of POLICY_FWD
// (early stop, KL coefficient, statistics) is taken by the gradient pass of
// POLICY_BWD itself (policy_rows_grad_kernel, dec_part)
static bool fused_decide(const smi_ppo_rnn_args& a, const RnnDims& d, const RnnScratch& s,
                         const Head& actor, int e) {
  // every gradient workgroup re-reduces the statistics pass's partials: only
  // while they are few (at 65536 segments, ~3000 partials per workgroup over
  // ~4000 workgroups took the gradient pass from 47 to 103 us)
  return a.mode != 0 && a.B_global == a.B && e < a.epoch_policy && fault() == 0 &&
         pol_stats_nb(a, d, s, actor) <= 512;
}

int ppo_rnn_phase(const smi_ppo_rnn_args& a, int phase, int e, hipStream_t st) {
  const RnnDims d = rnn_dims(a.B, a.T, a.horizon, a.obs_dim, a.rnn_hidden, a.h1, a.h2, a.act_dim,
                             a.critic_h1, a.critic_h2, a.pix_c, a.pix_h, a.pix_w, a.cnn_feat,
                             a.rnn_layer);
  const RnnScratch s = rnn_scratch(d, a.scratch);
  if (s.total_floats * 4 > a.scratch_bytes) return set_error(SMI_E_ARG, "ppo_rnn: scratch too small");
  const int* stop = s.ci + CI_STOP;
  const LstmP lm = lstm_params(a.lstm, d.Din, d.H);
  const float* cnn = a.lstm + d.nL;                    // stem = [lstm | cnn]
  const Head actor{a.actor, d.LA, d.Hin, d.h1, d.h2, d.A, 1};
  const Head critic{a.critic, d.LC, d.Hin, d.c1, d.c2, 1, 0};
  float* gA = a.xbuf;                                  // [actor head | lstm | cnn]
  float* gC = a.xbuf + d.nA_head + d.nS;               // [critic head | lstm | cnn]
  const int64_t NEg = (int64_t)d.E * a.B_global;
  switch (phase) {
    case SMI_RNN_PH_GAE: {
      int kt = ktime_begin(st);
      const int zrc = launch_zf_tmajor(a.obs, a.obs_next, d.B, d.T, d.S1, d.D, a.use_zf, a.zf_sum,
                                       a.zf_sumsq, a.zf_count, a.zf_eps, s.Xz, d.ldx, st, 0,
                                       d.F == 0);
      ktime_end(kt, KT_ZF_TMAJOR, 8.0 * (double)d.NG * d.D, st);      // read x, write z(x)
      RC(zrc);
      RC(cnn_features(a, d, cnn, d.S1, s.Xz, nullptr, s, st, nullptr));
      // the critic's LSTM pass over T + 1 steps (ppo.py:385) with the cell
      // states and gates of its first E steps kept: the first policy forward
      // (ppo.py:253-262 at epoch 0) is the same recurrence over the same
      // inputs from the same (h0, c0) with the same parameters, so
      // POLICY_FWD(0) reads these instead of recomputing them
      if (gae_prep_dual(a, d)) {
        // PREP's input (the reference z-filter over obs_iter), then both
        // recurrences in one launch: the critic's over T + 1 steps keeping E
        // steps' cells / gates, the reference policy's over E steps
        RC(launch_zf_tmajor(a.obs, a.obs_next, d.B, d.T, d.E, d.D, a.use_zf, a.rzf_sum,
                            a.rzf_sumsq, a.rzf_count, a.zf_eps, s.Xr, d.ldx, st, 0,
                            d.F == 0));
        const LstmP lc = lstm_layer(d, a.lstm, 0), lr = lstm_layer(d, a.ref_lstm, 0);
        LstmFwdArgs g0{nullptr, lc.Whh, lc.bhh, a.h0, a.c0, d.S1, d.B, d.H, hbuf_of(d, s, 0),
                       cbuf_of(d, s, 0), gates_of(d, s, 0), nullptr, s.Xz, d.ldx, d.Din, lc.Wih,
                       lc.bih, d.E};
        LstmFwdArgs g1{nullptr, lr.Whh, lr.bhh, a.h0, a.c0, d.E, d.B, d.H, s.hbufR, nullptr, nullptr,
                       nullptr, s.Xr, d.ldx, d.Din, lr.Wih, lr.bih, 0};
        RC(launch_lstm_fwd_x_dual(g0, g1, st));
      } else if (d.H > 0) {
        RC(lstm_forward(d, a.lstm, s.Xz, d.S1, a.h0, a.c0, s, true, st, nullptr, d.E));
      }
      RC(head_fwd(critic, head_in(d, s, s.Xz), d.Hld, d.NG, s.HA1, s.HA2, s.OUT, st, nullptr,
                  nullptr, nullptr, nullptr, 0.f, nullptr, nullptr, nullptr, false));
      hipLaunchKernelGGL(tmajor_to_bmajor_kernel, dim3(grid_of(d.NG)), dim3(kWG), 0, st, s.OUT,
                         d.S1, d.B, s.values, s.ci, s.cf);
      RC(check_launch("tmajor_to_bmajor_kernel"));
      int np = 0;
      kt = ktime_begin(st);
      RC(launch_gae_windows(s.values, nullptr, a.rewards, a.dones, d.B, d.T, d.Hz, a.gamma_tab,
                            a.lam_tab, a.gamma, a.gamma_H, s.adv, s.ret, s.gaepart, &np, st));
      // r, d (8 B) + V (4 (T+1)/T B) per env-step, adv + ret (8 B) per window
      ktime_end(kt, KT_GAE, (double)d.B * (8.0 * d.T + 4.0 * d.S1 + 8.0 * d.E), st);
      hipLaunchKernelGGL(reduce_partials_kernel, dim3(1), dim3(kWG), 0, st, s.gaepart, np, 2,
                         a.moments, nullptr, a.moments + 2, (double)d.NE);
      return check_launch("reduce_partials_kernel");
    }
    case SMI_RNN_PH_PREP: {
      // ref_pol (ppo.py:539): the reference model's forward over obs_iter.
      // With a.prep_independent != 0 it reads only the batch and the reference
      // parameters and writes only its own buffers (sp) and refmu, so the host
      // may run it on a second stream beside GAE (with its own smi_context).
      // With a.prep_independent == 0 it must follow GAE on the same stream: GAE
      // may have run its input transpose and recurrence (gae_prep_dual).
      RnnScratch sp = s;
      sp.xproj = s.xprojR; sp.hbuf = s.hbufR; sp.HA1 = s.HA1R; sp.HA2 = s.HA2R; sp.A2 = s.A2R;
      const float* X = s.Xr;
      if (!gae_prep_dual(a, d)) {   // (else the GAE phase ran this input and recurrence)
        RC(launch_zf_tmajor(a.obs, a.obs_next, d.B, d.T, d.E, d.D, a.use_zf, a.rzf_sum,
                            a.rzf_sumsq, a.rzf_count, a.zf_eps, s.Xr, d.ldx, st, 0,
                            d.F == 0));
        RC(cnn_features(a, d, a.ref_lstm + d.nL, d.E, s.Xr, nullptr, sp, st, nullptr));
        if (d.H > 0) RC(lstm_forward(d, a.ref_lstm, X, d.E, a.h0, a.c0, sp, false, st, nullptr));
      }
      const Head ref{a.ref_actor, d.LA, d.Hin, d.h1, d.h2, d.A, 1};
      return head_fwd(ref, head_in(d, sp, X), d.Hld, d.NE, sp.HA1, sp.HA2, s.refmu, st,
                      nullptr, nullptr, nullptr, nullptr, 0.f, nullptr, nullptr, nullptr, false);
    }
    case SMI_RNN_PH_POLICY_FWD: {
      if (e == 0) {
        launch_row_pack(d.A, d.NE, pol_rows(a, d, s), s.rowin, s.ret_tm, st);
        RC(check_launch("row_pack_kernel"));
      }
      if (e == 0 && (a.adv_out || a.ret_out)) {
        hipLaunchKernelGGL(adv_export_kernel, dim3(grid_of(d.NE)), dim3(kWG), 0, st,
                           pol_rows(a, d, s), a.adv_out, a.ret_out);
        RC(check_launch("adv_export_kernel"));
      }
      RC(cnn_features(a, d, cnn, d.E, s.Xz, s.A1, s, st, stop));
      if (d.H > 0 && e > 0) RC(lstm_forward(d, a.lstm, s.Xz, d.E, a.h0, a.c0, s, true, st, stop));
      PolRowArgs p = pol_rows(a, d, s);
      p.invN = (float)(1.0 / (double)NEg);
      const bool hs = pol_head_stats(a, d, s, actor);
      // (the KL check after the last update, e == epoch_policy, has no backward:
      // neither the activations nor the weight transposes are kept)
      const bool bwd_next = e < a.epoch_policy;
      RC(head_fwd(actor, head_in(d, s, s.Xz), d.Hld, d.NE, s.HA1, s.HA2, s.OUT, st, stop,
                  bwd_next ? s.wT : nullptr, nullptr, nullptr, 0.f, nullptr, hs ? &p : nullptr,
                  nullptr, bwd_next));
      const int nb = pol_stats_nb(a, d, s, actor);
      if (!hs) {
        const int kt = ktime_begin(st);
        if (a.mode == 0) launch_pol_stats<true>(d.A, nb, p, st);     // + the clip gradient
        else launch_pol_stats<false>(d.A, nb, p, st);
        // per row: mu, refmu, actions (3A) + adv, ret, bl, rbd (4) floats read
        ktime_end(kt, KT_POLICY_STATS, 4.0 * (double)d.NE * (3 * d.A + 4), st);
        RC(check_launch("policy_rows_stats_kernel"));
      }
      if (fused_decide(a, d, s, actor, e)) return SMI_OK;     // decided by POLICY_BWD's gradient pass
      if (a.B_global == a.B) {         // one rank: nothing to exchange before the decision
        DecideArgs da{a.pstat, e, a.epoch_policy, a.mode,
                      a.kl_target, a.kl_cutoff_coeff, NEg, a.hyper, a.actor + d.LA.flv, d.A,
                      c_entropy_of(d.A), s.ci, s.cf, a.stats};
        hipLaunchKernelGGL(reduce_decide_kernel, dim3(1), dim3(kWG), 0, st, s.part, nb, da, stop);
        return check_launch("reduce_decide_kernel");
      }
      hipLaunchKernelGGL(reduce_partials_kernel, dim3(1), dim3(kWG), 0, st, s.part, nb, PS_N,
                         a.pstat, stop, nullptr, 0.0);
      return check_launch("reduce_partials_kernel");
    }
    case SMI_RNN_PH_POLICY_DECIDE: {   // after the pstat all-reduce
      if (a.B_global == a.B) return SMI_OK;     // decided by POLICY_FWD's reduce_decide_kernel
      DecideArgs da{a.pstat, e, a.epoch_policy, a.mode,
                    a.kl_target, a.kl_cutoff_coeff, NEg, a.hyper, a.actor + d.LA.flv, d.A,
                    c_entropy_of(d.A), s.ci, s.cf, a.stats};
      hipLaunchKernelGGL(policy_decide_kernel, dim3(1), dim3(64), 0, st, da);
      return check_launch("policy_decide_kernel");
    }
    case SMI_RNN_PH_POLICY_BWD: {
      if (fault() == SMI_FAULT_POLICY_EPOCH_SHORT && e == a.epoch_policy - 1) return SMI_OK;
      PolRowArgs p = pol_rows(a, d, s);
      // clip: the log_var partials came from POLICY_FWD's fused pass, over its grid
      const int nb = a.mode == 0 ? pol_stats_blocks<true>(d.A, d.NE) : rnn_nblk(d.NE, kRowNT);
      if (fused_decide(a, d, s, actor, e)) {
        p.dec_part = s.part;
        p.dec_nb = pol_stats_nb(a, d, s, actor);
        p.dec = DecideArgs{a.pstat, e, a.epoch_policy, a.mode,
                           a.kl_target, a.kl_cutoff_coeff, NEg, a.hyper, a.actor + d.LA.flv, d.A,
                           c_entropy_of(d.A), s.ci, s.cf, a.stats};
      }
      // adapt: the gradient row pass as the fused head chain's prologue (one
      // launch fewer), or its own launch
      const bool pgh = pol_head_grad(a, d, s, actor);
      const int nb_pg = pgh ? head_bwd_blocks(d.NE) : nb;
      if (a.mode != 0 && !pgh) {     // clip: dz and the log_var partials came with POLICY_FWD's pass
        const int kt = ktime_begin(st);
        switch (d.A) {   // compile-time action widths 1..8 (registers); others generic
          case 1: hipLaunchKernelGGL((policy_rows_grad_kernel<kRowNT, 1>), dim3(nb), dim3(kRowNT), 0, st, p); break;
          case 2: hipLaunchKernelGGL((policy_rows_grad_kernel<kRowNT, 2>), dim3(nb), dim3(kRowNT), 0, st, p); break;
          case 3: hipLaunchKernelGGL((policy_rows_grad_kernel<kRowNT, 3>), dim3(nb), dim3(kRowNT), 0, st, p); break;
          case 4: hipLaunchKernelGGL((policy_rows_grad_kernel<kRowNT, 4>), dim3(nb), dim3(kRowNT), 0, st, p); break;
          case 5: hipLaunchKernelGGL((policy_rows_grad_kernel<kRowNT, 5>), dim3(nb), dim3(kRowNT), 0, st, p); break;
          case 6: hipLaunchKernelGGL((policy_rows_grad_kernel<kRowNT, 6>), dim3(nb), dim3(kRowNT), 0, st, p); break;
          case 7: hipLaunchKernelGGL((policy_rows_grad_kernel<kRowNT, 7>), dim3(nb), dim3(kRowNT), 0, st, p); break;
          case 8: hipLaunchKernelGGL((policy_rows_grad_kernel<kRowNT, 8>), dim3(nb), dim3(kRowNT), 0, st, p); break;
          default: hipLaunchKernelGGL((policy_rows_grad_kernel<kRowNT, 0>), dim3(nb), dim3(kRowNT), 0, st, p); break;
        }
        // per row: mu, refmu, actions (3A) + adv, bl (2) read, dz (A) written
        ktime_end(kt, KT_POLICY_GRAD, 4.0 * (double)d.NE * (4 * d.A + 2), st);
        RC(check_launch("policy_rows_grad_kernel"));
      }
      // the log_var gradient (and, fused, the clip-norm partials and the step
      // bump) as the dW reducer's epilogue task
      const bool fn = fused_clip_norm(a, d);
      DwEpilogue ex{};
      ex.lvpart = s.lvpart; ex.lv_nb = nb_pg; ex.lv_A = d.A;
      ex.lv = a.actor + d.LA.flv; ex.lv_out = gA + d.LA.flv;
      ex.skip = stop;
      if (fn) {
        ex.sq = s.part; ex.np = s.ci + CI_NP;
        ex.step = a.actor_step; ex.runs = s.ci + CI_RUNS;
      }
      return stem_backward(a, d, actor, lm, cnn, gA, s, d.nA_head, st, stop, &ex,
                           pgh ? &p : nullptr);
    }
    case SMI_RNN_PH_POLICY_APPLY: {
      if (fault() == SMI_FAULT_POLICY_EPOCH_SHORT && e == a.epoch_policy - 1) return SMI_OK;
      const int64_t n = d.nA_head + d.nS;
      const int g = grid_of(n, 1024);
      const int kt = ktime_begin(st);
      const bool fn = fused_clip_norm(a, d);
      if (!fn) {
        hipLaunchKernelGGL(sumsq_part_kernel, dim3(g), dim3(kWG), 0, st, gA, n, s.part, stop,
                           a.actor_step, s.ci + CI_RUNS);
        RC(check_launch("sumsq_part_kernel"));
      }
      AdamSplitArgs aa{a.actor, d.nA_head, a.lstm, d.nS, gA, a.actor_m, a.actor_v, a.actor_step,
                       a.hyper + SMI_HYP_LR_ACTOR, a.beta1, a.beta2, a.adam_eps, a.actor_wd,
                       a.clip_actor_grad ? a.actor_max_norm : 0.f, s.part, g, stop,
                       a.clip_actor_grad ? a.stats + SMI_ST_GRAD_NORM_ACTOR : nullptr, nullptr,
                       fn ? s.ci + CI_NP : nullptr};
      hipLaunchKernelGGL(adam_split_kernel, dim3(g), dim3(kWG), 0, st, aa);
      // grad-norm pass (g: 4 B) + Adam (p, g, m, v read 16 B; p, m, v written 12 B)
      ktime_end(kt, KT_ADAM, 32.0 * (double)n, st);
      return check_launch("adam_split_kernel");
    }
    case SMI_RNN_PH_VALUE_GRAD: {
      // value epoch 0: the last policy forward that ran (the KL check after
      // the last policy update, ppo.py:553-556, or the epoch-0 forward with
      // no update) left the stem's outputs, cell states, gates and conv
      // activations of exactly the current parameters: reused, not recomputed
      if (e > 0) {
        RC(cnn_features(a, d, cnn, d.E, s.Xz, s.A1, s, st, nullptr));
        if (d.H > 0) RC(lstm_forward(d, a.lstm, s.Xz, d.E, a.h0, a.c0, s, true, st, nullptr));
      }
      // dV = 2 (V - R) / N: written by the head forward's epilogue, except in
      // the last epoch, whose value_rows pass also sums the statistics of
      // ppo.py:324-331 (and on the layer-GEMM path)
      // (round 6: the last epoch's statistics too, one 5-double partial per
      // head workgroup, when the fused head runs and the partials fit s.part)
      const bool last = e == a.epoch_baseline - 1;
      const float vscale = (float)(2.0 / (double)NEg);
      bool vdone = false;
      const bool vstats = last && use_value_stats_head() &&
                          5 * (int64_t)head_bwd_blocks(d.NE) <= part_doubles(d);
      RC(head_fwd(critic, head_in(d, s, s.Xz), d.Hld, d.NE, s.HA1, s.HA2, s.OUT, st, nullptr,
                  s.wT, last && !vstats ? nullptr : s.ret_tm, last && !vstats ? nullptr : s.dOUT,
                  vscale, &vdone, nullptr, vstats ? s.part : nullptr));
      int nb = rnn_nblk((d.NE + 3) / 4, kRowNT);           // 4 rows per thread
      if (vdone && vstats) nb = head_bwd_blocks(d.NE);     // the head forward's partials
      if (!vdone) {
        const int kt = ktime_begin(st);
        hipLaunchKernelGGL(value_rows_kernel<kRowNT>, dim3(nb), dim3(kRowNT), 0, st, s.OUT, s.ret_tm, d.B,
                           d.E, vscale, s.dOUT, last ? s.part : nullptr);
        ktime_end(kt, KT_VALUE_ROWS, 12.0 * (double)d.NE, st);     // V, R read, dV written
        RC(check_launch("value_rows_kernel"));
      }
      if (last) {
        hipLaunchKernelGGL(reduce_partials_kernel, dim3(1), dim3(kWG), 0, st, s.part, nb, 5,
                           a.zbuf, nullptr, nullptr, 0.0);
        RC(check_launch("reduce_partials_kernel"));
      }
      if (!fused_clip_norm(a, d))
        return stem_backward(a, d, critic, lm, cnn, gC, s, d.nC_head, st, nullptr);
      DwEpilogue ex{};                // the clip-norm partials and the step bump
      ex.sq = s.part; ex.np = s.ci + CI_NP;
      ex.step = a.critic_step;
      return stem_backward(a, d, critic, lm, cnn, gC, s, d.nC_head, st, nullptr, &ex);
    }
    case SMI_RNN_PH_VALUE_APPLY: {
      if (fault() == SMI_FAULT_CRITIC_ADAM_SKIP) return SMI_OK;
      const int64_t nS = fault() == SMI_FAULT_CRITIC_STEM_OMIT ? 0 : d.nS;
      const int64_t n = d.nC_head + nS;
      const int g = grid_of(n, 1024);
      const int kt = ktime_begin(st);
      const bool fn = fused_clip_norm(a, d);
      if (!fn) {
        hipLaunchKernelGGL(sumsq_part_kernel, dim3(g), dim3(kWG), 0, st, gC, n, s.part, nullptr,
                           a.critic_step, nullptr);
        RC(check_launch("sumsq_part_kernel"));
      }
      AdamSplitArgs aa{a.critic, d.nC_head, a.lstm, nS, gC, a.critic_m, a.critic_v,
                       a.critic_step, a.hyper + SMI_HYP_LR_CRITIC, a.beta1, a.beta2, a.adam_eps,
                       a.critic_wd, a.clip_critic_grad ? a.critic_max_norm : 0.f, s.part, g,
                       nullptr, a.clip_critic_grad ? a.stats + SMI_ST_GRAD_NORM_CRITIC : nullptr,
                       nullptr, fn ? s.ci + CI_NP : nullptr};
      hipLaunchKernelGGL(adam_split_kernel, dim3(g), dim3(kWG), 0, st, aa);
      ktime_end(kt, KT_ADAM, 32.0 * (double)n, st);
      return check_launch("adam_split_kernel");
    }
    case SMI_RNN_PH_ZSTATS: {
      // zbuf (double) = [value sums (5) | column sums (D) | sums of squares (D)]
      if (!a.use_zf) return SMI_OK;
      // >= 64 rows per block (16 per wave, four in flight), at most 256 blocks
      const int nb = (int)std::max<int64_t>(1, std::min<int64_t>(256, (d.NE + 63) / 64));
      double* part = s.part;     // [nb][2][D] <= 65536 doubles for D <= 128
      if ((int64_t)nb * 2 * d.D > 4096 * 16) return set_error(SMI_E_ARG, "ppo_rnn: obs_dim too large");
      hipLaunchKernelGGL(obs_iter_colsum_kernel, dim3(nb), dim3(kWG), 0, st, a.obs, d.B, d.T, d.E,
                         d.D, part);
      RC(check_launch("obs_iter_colsum_kernel"));
      hipLaunchKernelGGL(reduce_partials_kernel, dim3(1), dim3(kWG), 0, st, part, nb, 2 * d.D,
                         a.zbuf + FS_Z, nullptr, nullptr, 0.0);
      return check_launch("reduce_partials_kernel");
    }
    case SMI_RNN_PH_ZAPPLY: {
      FinalArgs fa{a.zbuf, d.D, NEg, a.actor + d.LA.flv, d.A,
                   a.clip_critic_grad, a.zf_sum, a.zf_sumsq, a.zf_count, a.use_zf, a.stats, s.ci,
                   a.kl_record, a.kl_count, a.kl_capacity, a.epoch_policy};
      hipLaunchKernelGGL(rnn_final_kernel, dim3(1), dim3(64), 0, st, fa);
      return check_launch("rnn_final_kernel");
    }
    default:
      return set_error(SMI_E_ARG, "ppo_rnn: unknown phase");
  }
}

}  // namespace smi
