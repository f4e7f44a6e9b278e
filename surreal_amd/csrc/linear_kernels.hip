// linear_kernels.hip — layer-by-layer fp32 MFMA GEMMs for networks whose
// parameters do not fit one CU's LDS (PPO heads 300x200 over B*E rows, the
// LSTM input projection and weight gradients, DDPG actor 300x200 / critic
// 400x300; builders.py:35-175, ppo_net.py:137-152).  Every dense layer's
// forward, input-gradient and weight-gradient is the same LDS-tiled GEMM with
// a different operand view and epilogue:
//   fwd:  Y[m][n]  = act(b[n] + sum_k X[m][k] W[n][k])
//   dX:   dX[m][k] = mask(Xact[m][k] > 0) * sum_n dY[m][n] W[n][k]
//   dW:   dW[n][k] (+)= sum_m dY[m][n] X[m][k];  db[n] (+)= sum_m dY[m][n]
//         (db rides along as an extra all-ones column of X).  The reduction
//         over rows is split into KSPLIT slabs (dW is a 300x100 output over
//         ~20k rows: 10 tiles alone would leave 246 CUs idle); slab partials
//         go to the workspace and a fixed-order reducer adds them
//         (deterministic, no atomics).
// Tile 64x64, K-steps of 32, 256 threads: wave w owns rows [16w, 16w+16) x 64
// columns (4 accumulators of v_mfma_f32_16x16x4_f32).  The next K-step is
// loaded into registers while the current one runs on the MFMA pipe (LDS
// double buffer, one barrier per K-step).  LDS images follow the operand's
// contiguous dimension (leading dims 36 / 80: conflict-free MFMA operand
// reads and contiguous-dimension stores).  Global loads use clamped addresses
// and are zeroed afterwards (no predicated loads: see cdna_hip_programming.md).
#include <cmath>
#include <algorithm>
#include <stdlib.h>
#include <type_traits>
#include "smi_device.hpp"
#include "smi_internal.hpp"
#include "lstm_cell.hpp"

namespace smi {

enum { EPI_FWD = 0, EPI_DX = 1, EPI_DW = 2 };

constexpr int GBM = 64, GBN = 64, GBK = 32;
constexpr int LD_KC = 36;     // [row][k] images (k contiguous)
constexpr int LD_RC = 80;     // [k][row] images (row contiguous)
constexpr int G_STAGE = 2560; // floats per operand image per stage

struct GemmArgs {
  int M, N, K;
  // A(m,k) = A[m*a_rs + k*a_cs], B(k,n) = B[k*b_rs + n*b_cs]
  const float* A; int64_t a_rs, a_cs;
  const float* B; int64_t b_rs, b_cs;
  float* C; int64_t ldc;          // C[m*ldc + n]
  const float* bias;              // EPI_FWD
  int act;                        // EPI_FWD: ACT_*
  const float* mask; int64_t ldm; // EPI_DX: zero where mask[m*ldm+n] <= 0 (may be null)
  int accumulate;                 // EPI_DW (no split): C += result
  int ones_col;                   // EPI_DW: B(k, ones_col) == 1 (bias gradient column), -1 none
  float* bias_out;                // EPI_DW: column ones_col goes to bias_out[m]
  int kchunk;                     // K range of blockIdx.z: [z*kchunk, min(K, (z+1)*kchunk))
  float* part;                    // split-K partials [gridDim.z][M][N] (nullptr: no split)
  const int* skip;                // device flag: nonzero -> no-op (early stop)
  int avec, bvec;                 // 16-byte operand loads (set by gemm_launch)
  // EPI_DW with a two-source B (the LSTM's [x_t | h_{t-1}], one launch for the
  // W_ih and W_hh gradients): B2 != null makes columns n >= split_col read
  // B2[k*b2_rs + n - split_col] and land in C2 (ld ldc2); columns c1_real <= n
  // < split_col are padding (never stored); bias_out2 receives a copy of the
  // bias column (b_ih and b_hh have the same gradient).
  const float* B2; int64_t b2_rs; int split_col, c1_real;
  float* C2; int64_t ldc2; float* bias_out2;
  // EPI_FWD on the short-batch kernel: also C[m][N + j] = xsrc[m*xlds + j],
  // j < xcols (CriticNetworkX's cat(h1, action): the action block of the
  // next layer's input written by the layer that writes h1)
  const float* xsrc; int64_t xlds; int xcols;
};

// where output (m, n) of a weight gradient goes (bias column, the second
// destination of a two-source B, padding); returns the sum of squares of the
// values it stored (each destination element once: b_ih and b_hh both hold the
// bias gradient, so it counts twice, as in clip_grad_norm_ over both)
__device__ __forceinline__ float dw_put(const GemmArgs& g, int m, int n, float v) {
  if (n == g.ones_col) {
    const float b = g.accumulate ? g.bias_out[m] + v : v;
    g.bias_out[m] = b;
    if (g.bias_out2) {
      const float b2 = g.accumulate ? g.bias_out2[m] + v : v;
      g.bias_out2[m] = b2;
      return b * b + b2 * b2;
    }
    return b * b;
  }
  float* dst;
  if (g.B2 && n >= g.split_col) dst = g.C2 + (int64_t)m * g.ldc2 + (n - g.split_col);
  else if (g.B2 && n >= g.c1_real) return 0.f;               // padding column
  else dst = g.C + (int64_t)m * g.ldc + n;
  const float r = g.accumulate ? *dst + v : v;
  *dst = r;
  return r * r;
}

// Operand loader: one 64 (rows) x 32 (k) tile, 2048 elements, 8 per thread
// (scalar) or 2 float4 per thread (VEC: along the contiguous dimension, when
// that dimension's extent and the other stride are multiples of 4 and the base
// is 16-byte aligned — decided once per launch, a uniform branch).  Rows >=
// rdata and k >= kmax read as zero (clamped addresses, then masked); the
// all-ones column (dW bias gradient) is synthesised, never loaded.
struct TileRegs { float v[8]; };

// XCD-aware tile order (cdna_hip_programming.md T1): the dispatcher deals
// consecutive workgroups round-robin over the 8 XCDs (private L2 each); the
// bijective remap gives every XCD a contiguous run of the logical order, in
// which n-tiles of one m-tile (sharing A rows) and the tiles of one split-K
// slab (sharing the slab's rows of both operands) are neighbours.
struct TileIdx { int mt, nt, z; };
__device__ __forceinline__ TileIdx gemm_tile_index() {
  const int gm = gridDim.x, gn = gridDim.y;
  const int nwg = gm * gn * gridDim.z;
  const int orig = blockIdx.x + gm * (blockIdx.y + gn * blockIdx.z);
  int w = orig;
  if (nwg > 8) {
    const int x = orig & 7, q = nwg >> 3, r = nwg & 7;
    w = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (orig >> 3);
  }
  TileIdx t;
  t.nt = w % gn;
  t.mt = (w / gn) % gm;
  t.z = w / (gn * gm);
  return t;
}

template <bool KCONTIG>
__device__ __forceinline__ void gemm_load(const float* __restrict__ P, int64_t rs, int64_t cs,
                                          int r0, int rdata, int k0, int kmax, int ones_col,
                                          bool vec, TileRegs& t) {
  // interior tile (all 64 rows and 32 k valid, no synthesised column): plain
  // 16-byte loads, no clamps or masks
  if (vec && ones_col < 0 && r0 + 64 <= rdata && k0 + 32 <= kmax) {
    const float* base = KCONTIG ? P + (int64_t)r0 * rs + k0 : P + (int64_t)k0 * cs + r0;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int q = threadIdx.x + j * kWG;
      const float* src = KCONTIG ? base + (int64_t)(q >> 3) * rs + ((q & 7) << 2)
                                 : base + (int64_t)(q >> 4) * cs + ((q & 15) << 2);
      const float4 x = *reinterpret_cast<const float4*>(src);
      t.v[4 * j + 0] = x.x; t.v[4 * j + 1] = x.y; t.v[4 * j + 2] = x.z; t.v[4 * j + 3] = x.w;
    }
    return;
  }
  if (vec) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int q = threadIdx.x + j * kWG;
      if (KCONTIG) {            // 64 rows x 8 float4 along k
        const int r = q >> 3, k = (q & 7) << 2;
        const int rr = r0 + r, kk = k0 + k;
        const int rc = rr < rdata ? rr : rdata - 1;
        const int kc = kk < kmax ? kk : kmax - 4;
        const float4 x = *reinterpret_cast<const float4*>(P + (int64_t)rc * rs + kc);
        const bool ok = rr < rdata && kk < kmax;
        t.v[4 * j + 0] = ok ? x.x : 0.f; t.v[4 * j + 1] = ok ? x.y : 0.f;
        t.v[4 * j + 2] = ok ? x.z : 0.f; t.v[4 * j + 3] = ok ? x.w : 0.f;
      } else {                  // 32 k x 16 float4 along rows
        const int k = q >> 4, r = (q & 15) << 2;
        const int rr = r0 + r, kk = k0 + k;
        const int rc = rr < rdata ? rr : rdata - 4;
        const int kc = kk < kmax ? kk : kmax - 1;
        const float4 x = *reinterpret_cast<const float4*>(P + (int64_t)kc * cs + rc);
        const bool okk = kk < kmax, ok = okk && rr < rdata;
        t.v[4 * j + 0] = ok ? x.x : 0.f; t.v[4 * j + 1] = ok ? x.y : 0.f;
        t.v[4 * j + 2] = ok ? x.z : 0.f; t.v[4 * j + 3] = ok ? x.w : 0.f;
        if (ones_col >= 0 && okk) {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (rr + e == ones_col) t.v[4 * j + e] = 1.f;
        }
      }
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int idx = threadIdx.x + j * kWG;
    const int r = KCONTIG ? (idx >> 5) : (idx & 63);
    const int k = KCONTIG ? (idx & 31) : (idx >> 6);
    const int rr = r0 + r, kk = k0 + k;
    const int rc = rr < rdata ? rr : rdata - 1;
    const int kc = kk < kmax ? kk : kmax - 1;
    const float x = P[(int64_t)rc * rs + (int64_t)kc * cs];
    t.v[j] = (rr < rdata && kk < kmax) ? x : 0.f;
    if (ones_col >= 0 && rr == ones_col && kk < kmax) t.v[j] = 1.f;
  }
}

template <bool KCONTIG>
__device__ __forceinline__ void gemm_store(float* __restrict__ S, bool vec, const TileRegs& t) {
  if (vec) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int q = threadIdx.x + j * kWG;
      const float4 x = float4{t.v[4 * j], t.v[4 * j + 1], t.v[4 * j + 2], t.v[4 * j + 3]};
      if (KCONTIG) {
        const int r = q >> 3, k = (q & 7) << 2;
        *reinterpret_cast<float4*>(S + r * LD_KC + k) = x;
      } else {
        const int k = q >> 4, r = (q & 15) << 2;
        *reinterpret_cast<float4*>(S + k * LD_RC + r) = x;
      }
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int idx = threadIdx.x + j * kWG;
    const int r = KCONTIG ? (idx >> 5) : (idx & 63);
    const int k = KCONTIG ? (idx & 31) : (idx >> 6);
    if (KCONTIG) S[r * LD_KC + k] = t.v[j];
    else S[k * LD_RC + r] = t.v[j];
  }
}

// A is viewed with rows = m; B with rows = n (its "row" is the output column).
template <int EPI, bool AK, bool BK>
__global__ void __launch_bounds__(kWG)
gemm_kernel(GemmArgs g) {
  if (g.skip && g.skip[0] != 0) return;
  __shared__ __attribute__((aligned(16))) float sA[2][G_STAGE];
  __shared__ __attribute__((aligned(16))) float sB[2][G_STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, lk = lane >> 4;
  const TileIdx ti = gemm_tile_index();
  const int m0 = ti.mt * GBM, n0 = ti.nt * GBN;
  const int kb = ti.z * g.kchunk;
  const int ke = min(g.K, kb + g.kchunk);
  const int nk = (ke - kb + GBK - 1) / GBK;
  // B(k, n): viewed as rows n (B "row" stride b_cs), k stride b_rs
  f32x4 tot[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) tot[c] = f32x4{0.f, 0.f, 0.f, 0.f};
  // two K-steps of operands in flight in registers (R[0], R[1]) ahead of the
  // LDS double buffer: the global loads of step kt+2 are issued before step
  // kt's MFMAs, so each load has two compute phases to land
  TileRegs ra[2], rb[2];
  const int bdata = g.ones_col >= 0 ? g.ones_col : g.N;
  if (nk > 0) {
    gemm_load<AK>(g.A, g.a_rs, g.a_cs, m0, g.M, kb, ke, -1, g.avec, ra[0]);
    gemm_load<BK>(g.B, g.b_cs, g.b_rs, n0, bdata, kb, ke, g.ones_col, g.bvec, rb[0]);
  }
  if (nk > 1) {
    gemm_load<AK>(g.A, g.a_rs, g.a_cs, m0, g.M, kb + GBK, ke, -1, g.avec, ra[1]);
    gemm_load<BK>(g.B, g.b_cs, g.b_rs, n0, bdata, kb + GBK, ke, g.ones_col, g.bvec, rb[1]);
  }
  if (nk > 0) {
    gemm_store<AK>(sA[0], g.avec, ra[0]);
    gemm_store<BK>(sB[0], g.bvec, rb[0]);
  }
  __syncthreads();
  const int ar = wave * 16 + li;
  // one K-step from LDS image `cur`; register slot `cur` refills with step
  // kt+2, slot cur^1 (step kt+1) goes to the other LDS image afterwards.  The
  // loop is unrolled by two so the slots are compile-time registers.
  auto kstep = [&](int kt, auto cur_c) {
    constexpr int cur = decltype(cur_c)::value;
    if (kt + 2 < nk) {
      gemm_load<AK>(g.A, g.a_rs, g.a_cs, m0, g.M, kb + (kt + 2) * GBK, ke, -1, g.avec, ra[cur]);
      gemm_load<BK>(g.B, g.b_cs, g.b_rs, n0, bdata, kb + (kt + 2) * GBK, ke, g.ones_col, g.bvec,
                    rb[cur]);
    }
    const float* As = sA[cur];
    const float* Bs = sB[cur];
    // two-level accumulation: each K-step (32 products per output) starts a
    // fresh MFMA chain that is then added to the running sums — fp32 error of
    // a 32-term chain plus an nk-term chain instead of one 32*nk-term chain
    f32x4 acc[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[c] = f32x4{0.f, 0.f, 0.f, 0.f};
    // every operand of the K-step is read from LDS first, then 32 MFMAs run
    // back to back on 4 independent accumulator chains
    float av[8], bv[4][8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int k = 4 * u + lk;
      av[u] = AK ? As[ar * LD_KC + k] : As[k * LD_RC + ar];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int n = c * 16 + li;
        bv[c][u] = BK ? Bs[n * LD_KC + k] : Bs[k * LD_RC + n];
      }
    }
#pragma unroll
    for (int u = 0; u < 8; ++u)
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[c] = mfma4(av[u], bv[c][u], acc[c]);
#pragma unroll
    for (int c = 0; c < 4; ++c) tot[c] += acc[c];
    if (kt + 1 < nk) {
      gemm_store<AK>(sA[cur ^ 1], g.avec, ra[cur ^ 1]);
      gemm_store<BK>(sB[cur ^ 1], g.bvec, rb[cur ^ 1]);
    }
    __syncthreads();
  };
  for (int kt = 0; kt < nk; kt += 2) {
    kstep(kt, std::integral_constant<int, 0>{});
    if (kt + 1 < nk) kstep(kt + 1, std::integral_constant<int, 1>{});
  }
  // epilogue: 4 rows x 4 columns per lane, biases hoisted per column
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int n = n0 + c * 16 + li;
    if (n >= g.N) continue;
    float bias_n = 0.f;
    if constexpr (EPI == EPI_FWD) bias_n = g.bias ? g.bias[n] : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = m0 + wave * 16 + lk * 4 + i;
      if (m >= g.M) continue;
      float v = tot[c][i];
      if constexpr (EPI == EPI_FWD) {
        if (g.part) {                           // split-K slab: raw sums
          g.part[((int64_t)ti.z * g.M + m) * g.N + n] = v;
          continue;
        }
        v += bias_n;
        if (g.act == ACT_RELU) v = v > 0.f ? v : 0.f;
        else if (g.act == ACT_TANH) v = tanhf(v);
        g.C[(int64_t)m * g.ldc + n] = v;
      } else if constexpr (EPI == EPI_DX) {
        if (g.part) {                           // split-K slab: raw sums
          g.part[((int64_t)ti.z * g.M + m) * g.N + n] = v;
          continue;
        }
        if (g.mask) v = g.mask[(int64_t)m * g.ldm + n] > 0.f ? v : 0.f;
        g.C[(int64_t)m * g.ldc + n] = v;
      } else {
        if (g.part) {
          g.part[((int64_t)ti.z * g.M + m) * g.N + n] = v;
        } else if (n == g.ones_col) {
          g.bias_out[m] = g.accumulate ? g.bias_out[m] + v : v;
        } else {
          float* dst = g.C + (int64_t)m * g.ldc + n;
          *dst = g.accumulate ? *dst + v : v;
        }
      }
    }
  }
}

// zero row / ones vector selected by address (dwd_load, the reducers)
constexpr int DWD_ZMAX = 8192;
__device__ __attribute__((aligned(16))) float g_dwd_zero[DWD_ZMAX];
__device__ __attribute__((aligned(16))) float g_dwd_one[4] = {1.f, 0.f, 0.f, 0.f};

// split-K reducer: C[m][n] (+)= sum_z part[z][m][n]; the ones column goes to
// bias_out[m].  A workgroup owns 64 consecutive elements x 4 slab lanes: lane
// zl sums slabs zl, zl+4, ... with 4 independent accumulators (loads in
// flight), then the 4 lane sums are combined in LDS in a fixed order
// (deterministic, no atomics).
__global__ void __launch_bounds__(kWG)
gemm_splitk_reduce_kernel(const float* __restrict__ part, int S, GemmArgs g, const float* bias,
                          int act, const float* mask) {
  if (g.skip && g.skip[0] != 0) return;
  __shared__ float red[4][64];
  const int M = g.M, N = g.N;
  const int64_t MN = (int64_t)M * N;
  const int el = threadIdx.x & 63, zl = threadIdx.x >> 6;
  const int64_t e = (int64_t)blockIdx.x * 64 + el;
  const int64_t ec = e < MN ? e : MN - 1;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  int z = zl;
  if (S <= 64) {
    // every slab of the thread (z = zl + 4k) in flight at once, then the same
    // additions in the same order as the loop below (bit-identical): one
    // memory round trip instead of one per four slabs
    // (loads unconditional, slabs past S read a zero by address, and pinned
    // before the conditional adds below: with `zk < S ? load : 0` the compiler
    // sank each load into its own branch and waited on it there -- up to 16
    // round trips per block, round 6)
    // (addresses advanced by 4 slabs per k: the 64-bit index products per
    // load made the allocator reuse address registers and wait between loads)
    const float* pz = part + (int64_t)zl * MN + ec;
    const int64_t st4 = 4 * MN;
    float v[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) v[k] = *(zl + 4 * k < S ? pz + k * st4 : g_dwd_zero);
#pragma unroll
    for (int k = 0; k < 16; ++k) asm volatile("" : "+v"(v[k]));
    const int nfull = S > zl + 12 ? (S - zl - 12 + 15) / 16 : 0;   // z + 12 < S trips
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (j < nfull) {
        s0 += v[4 * j]; s1 += v[4 * j + 1]; s2 += v[4 * j + 2]; s3 += v[4 * j + 3];
      }
    }
#pragma unroll
    for (int k = 0; k < 16; ++k)
      if (k >= 4 * nfull && zl + 4 * k < S) s0 += v[k];
    z = S;
  }
  for (; z + 12 < S; z += 16) {
    s0 += part[(int64_t)z * MN + ec];
    s1 += part[(int64_t)(z + 4) * MN + ec];
    s2 += part[(int64_t)(z + 8) * MN + ec];
    s3 += part[(int64_t)(z + 12) * MN + ec];
  }
  for (; z < S; z += 4) s0 += part[(int64_t)z * MN + ec];
  red[zl][el] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (zl != 0 || e >= MN) return;
  float s = (red[0][el] + red[1][el]) + (red[2][el] + red[3][el]);
  const int m = (int)(e / N), n = (int)(e - (int64_t)m * N);
  if (bias) s += bias[n];                       // split-K forward epilogue
  if (act == ACT_RELU) s = s > 0.f ? s : 0.f;
  else if (act == ACT_TANH) s = tanhf(s);
  if (mask && !(mask[(int64_t)m * g.ldm + n] > 0.f)) s = 0.f;   // split-K input gradient
  dw_put(g, m, n, s);
}

// Small-K forward (K <= 64: the LSTM input projection x W_ih^T over the
// observation width, the first layer of the DDPG nets).  The tiled kernel is
// latency-bound there (two K-steps per 64x64 tile, prologue and epilogue
// dominate); this one stages the whole weight W[N][K] (zero-padded to 4*NKU
// k) in LDS once per workgroup, keeps a 64-row tile of X in registers as MFMA
// A operands, and sweeps all N columns in groups of four 16-column blocks
// (four independent NKU-long MFMA chains).  Workgroups are persistent over row
// tiles.
template <int NKU>
__global__ void __launch_bounds__(kWG)
gemm_smallk_fwd_kernel(const float* __restrict__ X, int64_t ldx, int M, int K,
                       const float* __restrict__ W, int64_t ldw, const float* __restrict__ bias,
                       int N, int act, float* __restrict__ Y, int64_t ldy, const int* skip) {
  if (skip && skip[0] != 0) return;
  extern __shared__ __attribute__((aligned(16))) float sW[];
  constexpr int LDK = 4 * NKU + 1;                  // odd: conflict-free B reads
  constexpr int LDO = 68;                           // output staging [16][68] per wave
  float* sb = sW + N * LDK;
  float* so = sb + ((N + 3) & ~3) + (threadIdx.x >> 6) * 16 * LDO;
  // staging: 8 independent loads in flight per thread (a plain loop waits for
  // each load before the next: ~80 serialised L2 round trips per thread)
  {
    const int tot = N * LDK;
    for (int e0 = threadIdx.x; e0 < tot; e0 += 8 * kWG) {
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int e = e0 + j * kWG;
        const int ec = e < tot ? e : tot - 1;
        const int n = ec / LDK, k = ec - n * LDK;
        const float x = W[(int64_t)n * ldw + (k < K ? k : K - 1)];
        v[j] = k < K ? x : 0.f;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int e = e0 + j * kWG;
        if (e < tot) sW[e] = v[j];
      }
    }
  }
  for (int n = threadIdx.x; n < N; n += kWG) sb[n] = bias ? bias[n] : 0.f;
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, li = lane & 15, lk = lane >> 4;
  const bool vec_out = ((reinterpret_cast<uintptr_t>(Y) & 15) == 0) && (ldy % 4 == 0);
  for (int tile = blockIdx.x; tile * 64 < M; tile += gridDim.x) {
    const int m = tile * 64 + wave * 16 + li;
    const int mc = m < M ? m : M - 1;
    float a[NKU];
#pragma unroll
    for (int u = 0; u < NKU; ++u) {
      const int k = 4 * u + lk;
      const float x = X[(int64_t)mc * ldx + (k < K ? k : K - 1)];
      a[u] = k < K ? x : 0.f;
    }
    for (int nb = 0; nb < N; nb += 64) {
      f32x4 acc[4];
      const float* w[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        acc[c] = f32x4{0.f, 0.f, 0.f, 0.f};
        const int n = nb + c * 16 + li;
        w[c] = sW + (n < N ? n : N - 1) * LDK + lk;
      }
      // all B operands of the group first (one LDS round trip), then the MFMAs
      float bw[4][NKU];
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int u = 0; u < NKU; ++u) bw[c][u] = w[c][4 * u];
#pragma unroll
      for (int u = 0; u < NKU; ++u)
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[c] = mfma4(a[u], bw[c][u], acc[c]);
      // epilogue through the wave's LDS slab: rows leave as 16-byte stores
      // (a wave-instruction writes 4 rows x 256 contiguous bytes)
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int col = nb + c * 16 + li;
        const float bn = col < N ? sb[col] : 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          float v = acc[c][i] + bn;
          if (act == ACT_RELU) v = v > 0.f ? v : 0.f;
          else if (act == ACT_TANH) v = tanhf(v);
          so[(lk * 4 + i) * LDO + c * 16 + li] = v;
        }
      }
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int r = j * 4 + (lane >> 4), c4 = (lane & 15) * 4;
        const int row = tile * 64 + wave * 16 + r, col = nb + c4;
        const float4 v = *reinterpret_cast<const float4*>(so + r * LDO + c4);
        if (row < M) {
          float* dst = Y + (int64_t)row * ldy + col;
          if (vec_out && col + 3 < N) {
            *reinterpret_cast<float4*>(dst) = v;
          } else {
            if (col < N) dst[0] = v.x;
            if (col + 1 < N) dst[1] = v.y;
            if (col + 2 < N) dst[2] = v.z;
            if (col + 3 < N) dst[3] = v.w;
          }
        }
      }
      __builtin_amdgcn_wave_barrier();
    }
  }
}

static int launch_smallk_fwd(const float* X, int64_t ldx, int M, int K, const float* W,
                             int64_t ldw, const float* b, int N, int act, float* Y, int64_t ldy,
                             hipStream_t st, const int* skip) {
  const int nku = (K + 3) / 4 <= 4 ? 4 : (K + 3) / 4 <= 8 ? 8 : (K + 3) / 4 <= 12 ? 12 : 16;
  const size_t lds = ((size_t)N * (4 * nku + 1) + ((N + 3) & ~3) + 4 * 16 * 68) * 4;
  const int tiles = (M + 63) / 64;
  const int kslot = ktime_begin(st);
#define SMI_SK_CASE(V)                                                                         \
  if (nku == V) {                                                                              \
    auto k = gemm_smallk_fwd_kernel<V>;                                                        \
    allow_lds(k, lds);                                                                         \
    static int cap = 0;                                                                        \
    if (!cap) cap = resident_grid(k, kWG, lds);                                                \
    const int grid = tiles < cap ? tiles : cap;                                                \
    hipLaunchKernelGGL(k, dim3(grid), dim3(kWG), lds, st, X, ldx, M, K, W, ldw, b, N, act, Y, \
                       ldy, skip);                                                             \
  }
  SMI_SK_CASE(4) SMI_SK_CASE(8) SMI_SK_CASE(12) SMI_SK_CASE(16)
#undef SMI_SK_CASE
  ktime_end(kslot, KT_GEMM_FWD, 2.0 * M * (double)N * K, st);
  return check_launch("gemm_smallk_fwd_kernel");
}

// Weight-gradient GEMM with 128x128 output tiles (dW[m][n] = sum_r dY[r][m]
// X[r][n], r = the B*E rows).  The 64x64 kernel re-reads dY once per 64
// output columns and X once per 64 output rows (5x / 4x for the 300x200
// head): at these shapes the launch moves ~5x its unique bytes through L2 and
// is bound by that, not by the MFMAs.  128x128 halves both re-read factors
// and raises MFMAs per LDS operand read (16 MFMAs per 10 reads).  Both
// operands are row-contiguous slabs of 32 rows: float4 loads straight into
// [k][col] LDS images (row pitch 144: a half-wave's 32 lanes hit 32 banks),
// one K-step of register prefetch, one barrier per K-step.  Wave w owns
// output rows [32w, 32w+32) x 128 columns (16 accumulators).  The reduction
// is one MFMA chain per K-slab (split-K keeps slabs <= 512 rows); slab
// partials go to the fixed-order reducer as in gemm_kernel.
constexpr int D2_T = 128, D2_LD = 144;

__device__ __forceinline__ void dw2_load(const float* __restrict__ P, int64_t rs, int c0,
                                         int cdata, int ones_col, int k0, int kmax, float4 (&r)[4]) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int q = threadIdx.x + j * kWG;            // 32 rows x 32 float4
    const int k = q >> 5, c = c0 + ((q & 31) << 2);
    const int kk = k0 + k;
    const int kc = kk < kmax ? kk : kmax - 1;
    const int cc = c + 3 < cdata ? c : (cdata >= 4 ? cdata - 4 : 0);
    float4 v = *reinterpret_cast<const float4*>(P + (int64_t)kc * rs + cc);
    const bool okk = kk < kmax;
    v.x = okk && c < cdata ? v.x : 0.f;
    v.y = okk && c + 1 < cdata ? v.y : 0.f;
    v.z = okk && c + 2 < cdata ? v.z : 0.f;
    v.w = okk && c + 3 < cdata ? v.w : 0.f;
    if (ones_col >= 0 && okk) {
      if (c == ones_col) v.x = 1.f;
      if (c + 1 == ones_col) v.y = 1.f;
      if (c + 2 == ones_col) v.z = 1.f;
      if (c + 3 == ones_col) v.w = 1.f;
    }
    r[j] = v;
  }
}

__device__ __forceinline__ void dw2_store(float* __restrict__ S, const float4 (&r)[4]) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int q = threadIdx.x + j * kWG;
    *reinterpret_cast<float4*>(S + (q >> 5) * D2_LD + ((q & 31) << 2)) = r[j];
  }
}

__global__ void __launch_bounds__(kWG)
gemm_dw128_kernel(GemmArgs g) {
  if (g.skip && g.skip[0] != 0) return;
  __shared__ __attribute__((aligned(16))) float sA[2][32 * D2_LD];
  __shared__ __attribute__((aligned(16))) float sB[2][32 * D2_LD];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, lk = lane >> 4;
  const TileIdx ti = gemm_tile_index();
  const int m0 = ti.mt * D2_T, n0 = ti.nt * D2_T;
  const int kb = ti.z * g.kchunk;
  const int ke = min(g.K, kb + g.kchunk);
  const int nk = (ke - kb + 31) / 32;
  const int bdata = g.ones_col >= 0 ? g.ones_col + 1 : g.N;   // the ones column is synthesised
  const int bload = g.ones_col >= 0 ? g.ones_col : g.N;       // real columns of X
  f32x4 acc[2][8];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 8; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  float4 ra[4], rb[4];
  (void)bdata;
  if (nk > 0) {
    dw2_load(g.A, g.a_cs, m0, g.M, -1, kb, ke, ra);
    dw2_load(g.B, g.b_rs, n0, bload, g.ones_col, kb, ke, rb);
    dw2_store(sA[0], ra);
    dw2_store(sB[0], rb);
  }
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) {
      dw2_load(g.A, g.a_cs, m0, g.M, -1, kb + (kt + 1) * 32, ke, ra);
      dw2_load(g.B, g.b_rs, n0, bload, g.ones_col, kb + (kt + 1) * 32, ke, rb);
    }
    const float* As = sA[cur];
    const float* Bs = sB[cur];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int kr = (4 * u + lk) * D2_LD;
      float av[2], bv[8];
#pragma unroll
      for (int a = 0; a < 2; ++a) av[a] = As[kr + wave * 32 + a * 16 + li];
#pragma unroll
      for (int b = 0; b < 8; ++b) bv[b] = Bs[kr + b * 16 + li];
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 8; ++b) acc[a][b] = mfma4(av[a], bv[b], acc[a][b]);
    }
    if (kt + 1 < nk) {
      dw2_store(sA[cur ^ 1], ra);
      dw2_store(sB[cur ^ 1], rb);
    }
    __syncthreads();
  }
#pragma unroll
  for (int b = 0; b < 8; ++b) {
    const int n = n0 + b * 16 + li;
    if (n >= g.N) continue;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = m0 + wave * 32 + a * 16 + lk * 4 + i;
        if (m >= g.M) continue;
        const float v = acc[a][b][i];
        if (g.part) {
          g.part[((int64_t)ti.z * g.M + m) * g.N + n] = v;
        } else if (n == g.ones_col) {
          g.bias_out[m] = g.accumulate ? g.bias_out[m] + v : v;
        } else {
          float* dst = g.C + (int64_t)m * g.ldc + n;
          *dst = g.accumulate ? *dst + v : v;
        }
      }
  }
}

// Weight gradient with operands straight from global memory into MFMA
// registers (no LDS staging, no barriers in the main loop).  dW[m][n] =
// sum_r dY[r][m] * X[r][n] reduces over the rows, which is the MFMA k index;
// a 16x16x4 MFMA's A operand for lane (li, lk) is (row lk, column li) and its
// B operand (row lk, column li), so one wave loads a 4-row step of BOTH
// operands as row-contiguous vectors: lane li takes MT consecutive dY columns
// m0 + MT*li + t (one per MFMA m-tile t) and 4 consecutive X columns per
// 64-column half, i.e. 16-byte loads that feed MT x NT MFMAs.  The output
// columns are thereby interleaved across tiles; the epilogue undoes that.  The
// four waves of a workgroup take interleaved 4-row steps of one row slab (P
// steps prefetched in registers) and are combined through LDS in a fixed
// order; slabs go to the split-K partials.  Row-major dY/X of the heads, the
// LSTM input/recurrent weights and the DDPG nets all take this path.
#ifndef SMI_DWD_DIAG
#define SMI_DWD_DIAG 0
#endif
// per-workgroup clock trace of the grouped launch (bench_dwgroup only; the
// `dwtrace` builds), independent of the DIAG mode
#ifndef SMI_DWD_TRACE
#define SMI_DWD_TRACE (SMI_DWD_DIAG == 3)
#endif
#ifndef SMI_DWD_P
#define SMI_DWD_P 4
#endif
#ifndef SMI_DWD_OCC
#define SMI_DWD_OCC 2
#endif
constexpr int DWD_P = SMI_DWD_P;   // steps in flight per wave

// Rows past the slab and the synthesised bias column are selected by ADDRESS
// (a zero row / a {1, 0, 0, 0} vector in device memory), never by masking the
// loaded value: the loads then feed the MFMAs untouched and the compiler keeps
// all P steps in flight.  Columns past M / N read clamped addresses; they only
// reach outputs the epilogue drops.

template <int MT, int NT, bool VA, bool VB, int NB = NT>
__device__ __forceinline__ void dwd_load(const GemmArgs& g, int r, int ke, int m0, int n0, int bdata,
                                         float (&av)[MT], float (&bv)[NT]) {
  const int li = threadIdx.x & 15;
  const bool ok = r < ke;
  const float* Ar = ok ? g.A + (int64_t)r * g.a_cs : g_dwd_zero;
  const float* Br = ok ? g.B + (int64_t)r * g.b_rs : g_dwd_zero;
  // second source (columns >= split_col): its row base, shifted so that column
  // cb reads Br2 + cb (rows past the slab read the zero row at offset cb - split)
  const float* Br2 = g.B2 ? (ok ? g.B2 + (int64_t)r * g.b2_rs - g.split_col
                                : g_dwd_zero - g.split_col)
                          : Br;
  const int split = g.B2 ? g.split_col : 0x7fffffff;
  const float* one = ok ? g_dwd_one : g_dwd_zero;
  if constexpr (MT == 4 && VA) {
    const int c = min(m0 + 4 * li, g.M - 4);
    const float4 x = *reinterpret_cast<const float4*>(Ar + c);
    av[0] = x.x; av[1] = x.y; av[2] = x.z; av[3] = x.w;
  } else {
#pragma unroll
    for (int t = 0; t < MT; ++t) av[t] = Ar[min(m0 + MT * li + t, g.M - 1)];
  }
#pragma unroll
  for (int h = 0; h < NB / 4; ++h) {
    const int cb = n0 + 64 * h + 4 * li;
    if constexpr (VB) {
      const float* src = cb < bdata ? (cb >= split ? Br2 : Br) + cb
                                    : (cb == g.ones_col ? one : g_dwd_zero);
      const float4 x = *reinterpret_cast<const float4*>(src);
      bv[4 * h] = x.x; bv[4 * h + 1] = x.y; bv[4 * h + 2] = x.z; bv[4 * h + 3] = x.w;
    } else {
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int c = cb + t;
        bv[4 * h + t] = *(c < bdata ? (c >= split ? Br2 : Br) + c
                                    : (c == g.ones_col ? one : g_dwd_zero));
      }
    }
  }
}

// Unchecked streaming loop over a slab whose rows are all valid (every slab
// but possibly the last: slab lengths are multiples of the prefetch window)
// with 16-byte operands: the lane's operand addresses are formed once and
// advanced by RS rows per step, so a step is its loads and MFMAs only — no
// per-step 64-bit row products, clamps, zero-row selects or exec-masked
// branches (the checked loop spends ~40 VALU/SALU ops per step on them).
// The last DWD_P steps are peeled without loads (no reads past the slab).
// Same MFMA chains in the same order as the checked loop: bit-identical.
#ifndef SMI_DWD_FAST
#define SMI_DWD_FAST 1
#endif
__device__ __forceinline__ bool use_dwd_fast() { return SMI_DWD_FAST != 0; }

template <int MT, int NT, int NB, int RS>
__device__ __forceinline__ void dwd_main_fast(const GemmArgs& g, int rw, int nsteps, int m0, int n0,
                                              int bdata, f32x4 (&acc)[MT][NT]) {
  static_assert(MT == 4 || MT == 1, "fast dW loop: 4 m sub-tiles (float4 A) or 1 (scalar A)");
  constexpr int NH = NB / 4;
  const int li = threadIdx.x & 15;
  const float* pa = g.A + (int64_t)rw * g.a_cs + (MT == 4 ? min(m0 + 4 * li, g.M - 4)
                                                          : min(m0 + li, g.M - 1));
  const int64_t sa = (int64_t)RS * g.a_cs;
  const float* pb[NH];
  int64_t sb[NH];
#pragma unroll
  for (int h = 0; h < NH; ++h) {
    const int cb = n0 + 64 * h + 4 * li;
    if (cb < bdata) {
      if (g.B2 && cb >= g.split_col) {
        pb[h] = g.B2 + (int64_t)rw * g.b2_rs + (cb - g.split_col);
        sb[h] = (int64_t)RS * g.b2_rs;
      } else {
        pb[h] = g.B + (int64_t)rw * g.b_rs + cb;
        sb[h] = (int64_t)RS * g.b_rs;
      }
    } else {
      pb[h] = cb == g.ones_col ? g_dwd_one : g_dwd_zero;
      sb[h] = 0;
    }
  }
  float4 av[DWD_P], bv[DWD_P][NH];
  // global (addrspace 1) loads spelled out: with the prologue pinned below the
  // compiler no longer infers the address space and emits flat loads, which
  // also count against lgkmcnt
  using gf4 = const __attribute__((address_space(1))) f32x4;
  using gf1 = const __attribute__((address_space(1))) float;
  auto f4 = [](const f32x4 x) { return float4{x[0], x[1], x[2], x[3]}; };
  auto load = [&](int p) {
    if constexpr (MT == 4) av[p] = f4(*(gf4*)pa);
    else av[p].x = *(gf1*)pa;
    pa += sa;
#pragma unroll
    for (int h = 0; h < NH; ++h) {
      bv[p][h] = f4(*(gf4*)pb[h]);
      pb[h] += sb[h];
    }
  };
  auto step = [&](int p) {
    const float a4[4] = {av[p].x, av[p].y, av[p].z, av[p].w};
#if SMI_DWD_DIAG == 2
    // diagnostic (bench_dwgroup A/B only): the operand stream without the MFMAs
    acc[0][0][0] += (a4[0] + a4[1]) + (a4[2] + a4[3]);
#pragma unroll
    for (int h = 0; h < NH; ++h) acc[0][0][1] += (bv[p][h].x + bv[p][h].y) + (bv[p][h].z + bv[p][h].w);
#else
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const float4 q = bv[p][b >> 2];
      const float bb = (b & 3) == 0 ? q.x : (b & 3) == 1 ? q.y : (b & 3) == 2 ? q.z : q.w;
#pragma unroll
      for (int a = 0; a < MT; ++a) acc[a][b] = mfma4(a4[a], bb, acc[a][b]);
    }
#endif
  };
  // the prologue's loads are pinned in step order too: the loop header's
  // vmcnt is the merge of the preheader and the back edge, so one prologue
  // load issued out of order (the scheduler put b0 seventh of eight) made
  // every iteration wait at vmcnt(1), i.e. on the loads just issued
#pragma unroll
  for (int p = 0; p < DWD_P; ++p) {
    load(p);
    __builtin_amdgcn_sched_barrier(0);
  }
  // sched_barrier pins each refill right behind the MFMAs of the step it
  // replaces: without it the scheduler sinks all DWD_P refills to the end of
  // the unrolled body and the next iteration waits on them (vmcnt(9..0)), i.e.
  // no prefetch distance at all
  // 16-wide tail tiles (MT == 1) run the longest slabs of a balanced grouped
  // launch (~2.5x the rows of a full tile's slab): their MFMA chain restarts
  // every DWD_P steps and the blocks are summed in a second register set, so
  // a wave's fp32 chain is DWD_P + steps / DWD_P long instead of steps long
  // (the value head's 1-row gradient sums 21504 rows with heavy cancellation)
  f32x4 tot[MT][NT];
  if constexpr (MT == 1) {
#pragma unroll
    for (int b = 0; b < NT; ++b) tot[0][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  for (int s0 = DWD_P; s0 < nsteps; s0 += DWD_P) {
#pragma unroll
    for (int p = 0; p < DWD_P; ++p) {
      step(p);
      // diagnostic SMI_DWD_DIAG 1 (bench_dwgroup A/B only): the MFMAs without
      // the operand stream (the first DWD_P steps' operands reused)
      if constexpr (SMI_DWD_DIAG != 1) load(p);
      __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (MT == 1) {
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        tot[0][b] += acc[0][b];
        acc[0][b] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
  }
#pragma unroll
  for (int p = 0; p < DWD_P; ++p) step(p);
  if constexpr (MT == 1) {
#pragma unroll
    for (int b = 0; b < NB; ++b) acc[0][b] = tot[0][b] + acc[0][b];
  }
}

// WV waves per workgroup (4: one per SIMD; 8: two per SIMD, each wave takes
// every WV-th 4-row step of the slab, so a SIMD interleaves two waves' loads
// and MFMAs; the waves' sums meet in LDS in a fixed tree order)
template <int MT, int NT, bool VA, bool VB, int WV>
__device__ __forceinline__ void dwd_tile(const GemmArgs& g, const TileIdx ti, float4* dwd_red) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int li = lane & 15, lk = lane >> 4;
  const int m0 = ti.mt * 16 * MT, n0 = ti.nt * 16 * NT;
  const int kb = ti.z * g.kchunk;
  const int ke = min(g.K, kb + g.kchunk);
  constexpr int RS = 4 * WV;                      // rows per step of the workgroup
  const int nsteps = (ke - kb + RS - 1) / RS;
  const int bdata = g.ones_col >= 0 ? g.ones_col : g.N;
  const int rw = kb + 4 * wave + lk;              // this lane's row in step 0
  f32x4 acc[MT][NT];
#pragma unroll
  for (int a = 0; a < MT; ++a)
#pragma unroll
    for (int b = 0; b < NT; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  // loads are unconditional (rows past the slab read clamped and zeroed) so
  // the compiler's vmcnt waits stay partial across the unrolled P steps;
  // slabs are multiples of 4*WV*P rows, only the last one runs zero steps
  // NB of the NT column sub-tiles carry data: a tile whose upper 64-column
  // half lies past N (e.g. columns 320..383 of a 301-wide gradient) runs the
  // half-width loop (wave-uniform choice, no loads or MFMAs for that half)
  auto mainloop = [&](auto nbc) {
    constexpr int NB = decltype(nbc)::value;
    float av[DWD_P][MT], bv[DWD_P][NT];
#pragma unroll
    for (int p = 0; p < DWD_P; ++p)
      dwd_load<MT, NT, VA, VB, NB>(g, rw + RS * p, ke, m0, n0, bdata, av[p], bv[p]);
    for (int s0 = 0; s0 < nsteps; s0 += DWD_P) {
#pragma unroll
      for (int p = 0; p < DWD_P; ++p) {
#pragma unroll
        for (int b = 0; b < NB; ++b)
#pragma unroll
          for (int a = 0; a < MT; ++a) acc[a][b] = mfma4(av[p][a], bv[p][b], acc[a][b]);
        dwd_load<MT, NT, VA, VB, NB>(g, rw + RS * (s0 + p + DWD_P), ke, m0, n0, bdata, av[p], bv[p]);
        __builtin_amdgcn_sched_barrier(0);     // keep the refill here (see dwd_main_fast)
      }
    }
  };
  // full slabs of 16-byte operands take the unchecked streaming loop
  // (MT == 1: scalar A loads, no A alignment needed)
  constexpr bool kFast = VB && ((VA && MT == 4) || MT == 1);
  bool fast = false;
  if constexpr (kFast)
    fast = use_dwd_fast() && nsteps >= DWD_P && nsteps % DWD_P == 0 && kb + nsteps * RS <= ke;
  constexpr int NBH = NT > 4 ? 4 : NT;
  if (NT == 8 && n0 + 64 >= g.N) {
    if constexpr (kFast) {
      if (fast) dwd_main_fast<MT, NT, NBH, RS>(g, rw, nsteps, m0, n0, bdata, acc);
      else mainloop(std::integral_constant<int, NBH>{});
    } else {
      mainloop(std::integral_constant<int, NBH>{});
    }
  } else {
    if constexpr (kFast) {
      if (fast) dwd_main_fast<MT, NT, NT, RS>(g, rw, nsteps, m0, n0, bdata, acc);
      else mainloop(std::integral_constant<int, NT>{});
    } else {
      mainloop(std::integral_constant<int, NT>{});
    }
  }
  // combine the waves in a fixed tree: at stride h, waves [h, 2h) add into
  // waves [0, h), two at a time through the two LDS buffers (WV = 4 gives
  // (w0 + w2) + (w1 + w3))
  auto put = [&](float4* buf) {
#pragma unroll
    for (int a = 0; a < MT; ++a)
#pragma unroll
      for (int b = 0; b < NT; ++b) {
        const f32x4 v = acc[a][b];
        buf[(a * NT + b) * 64 + lane] = float4{v[0], v[1], v[2], v[3]};
      }
  };
  auto add = [&](const float4* buf) {
#pragma unroll
    for (int a = 0; a < MT; ++a)
#pragma unroll
      for (int b = 0; b < NT; ++b) {
        const float4 v = buf[(a * NT + b) * 64 + lane];
        acc[a][b] += f32x4{v.x, v.y, v.z, v.w};
      }
  };
#pragma unroll
  for (int h = WV / 2; h >= 1; h >>= 1) {
#pragma unroll
    for (int c = 0; c < h; c += 2) {
      if (wave >= h + c && wave < h + c + 2) put(dwd_red + (wave - h - c) * MT * NT * 64);
      __syncthreads();
      if (wave >= c && wave < c + 2 && wave < h) add(dwd_red + (wave - c) * MT * NT * 64);
      __syncthreads();
    }
  }
  if (wave != 0) return;
  // D(row lk*4+i, col li) of tile (a, b) is dW[m][n] with
  // m = m0 + MT*(lk*4+i) + a, n = n0 + 64*(b/4) + 4*li + b%4
  const bool vec_part = g.part && (g.N & 3) == 0;
#pragma unroll
  for (int a = 0; a < MT; ++a)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = m0 + MT * (lk * 4 + i) + a;
      if (m >= g.M) continue;
#pragma unroll
      for (int h = 0; h < NT / 4; ++h) {
        const int nb = n0 + 64 * h + 4 * li;
        if (vec_part) {
          if (nb < g.N)
            *reinterpret_cast<float4*>(g.part + ((int64_t)ti.z * g.M + m) * g.N + nb) =
                float4{acc[a][4 * h][i], acc[a][4 * h + 1][i], acc[a][4 * h + 2][i],
                       acc[a][4 * h + 3][i]};
          continue;
        }
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const int n = nb + t;
          if (n >= g.N) continue;
          const float v = acc[a][4 * h + t][i];
          if (g.part) g.part[((int64_t)ti.z * g.M + m) * g.N + n] = v;
          else dw_put(g, m, n, v);
        }
      }
    }
}

template <int MT, int NT, bool VA, bool VB, int WV>
__global__ void __launch_bounds__(64 * WV, WV == 4 ? SMI_DWD_OCC : 1)
gemm_dwd_kernel(GemmArgs g) {
  if (g.skip && g.skip[0] != 0) return;
  extern __shared__ float4 dwd_red[];            // 2 x [MT*NT][64] float4
  dwd_tile<MT, NT, VA, VB, WV>(g, gemm_tile_index(), dwd_red);
}

// Grouped weight gradients: every dW GEMM of one backward phase (the head's
// three layers and the LSTM's fused W_ih | W_hh) in ONE launch.  Workgroups are
// dealt to GEMMs by a prefix over their (tiles x slabs); slab lengths are
// balanced so every workgroup reduces about the same number of rows; each GEMM
// writes its own split-K partials, and one grouped reducer finishes them all.
// One launch and one reduce per phase instead of a launch + reduce per layer
// (and no side stream): the ~20 us fixed cost of a dW launch is paid once.
constexpr int kDwGroupMax = 8;   // entries of one reducer (two launches' worth)
constexpr int kDwSplitMax = 6;    // entries of one grouped launch after tail splits
struct DwGroup {
  DwEpilogue x;                  // optional epilogue task of the reducer (smi_internal.hpp)
  GemmArgs g[kDwGroupMax];
  int wg0[kDwGroupMax + 1];      // workgroup prefix
  int rb0[kDwGroupMax + 1];      // reducer-block prefix
  int gm[kDwGroupMax], gn[kDwGroupMax], S[kDwGroupMax];
  int vec[kDwGroupMax];          // 2*VA + VB
  int narrow[kDwGroupMax];       // last m-tile is a 16-wide tail (M % 64 in 1..16)
  int n;
};

// output tile width of the grouped launch in 16-column sub-tiles, and its
// occupancy.  Measured (C3 bench, one MI355X, interleaved trials): 64 x 64
// tiles at 3 waves per SIMD (130 VGPRs) 120.5 us per grouped launch (0.336 of
// the f32 MFMA peak), learn 8.21 ms, against 64 x 128 tiles at 2 waves per
// SIMD (222 VGPRs) 129.6 us, 8.46 ms: the third wave hides more of the
// operand-stream latency (the launch waits on memory ~60 % of its wave
// cycles, PMC SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES) than the halved MFMA reuse
// per loaded byte costs.
#ifndef SMI_DWG_NT
#define SMI_DWG_NT 4
#endif
#ifndef SMI_DWG_OCC
#define SMI_DWG_OCC (SMI_DWG_NT == 4 ? 3 : 2)
#endif
constexpr int DWG_NT = SMI_DWG_NT;

#if SMI_DWD_TRACE
// diagnostic (bench_dwgroup only): per-workgroup {start, end, HW_ID, XCC_ID |
// group << 8} in 100 MHz wall-clock ticks plus {start, end} of the shader
// clock (clock64: the in-kernel clock is its delta over the wall delta),
// read back by smi_diag_dw_trace
constexpr int kDwTraceMax = 8192;
__device__ unsigned long long g_dw_trace[kDwTraceMax][6];
extern "C" int smi_diag_dw_trace(void* dst, int n) {
  if (n > kDwTraceMax) n = kDwTraceMax;
  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_dw_trace), (size_t)n * 48, 0, hipMemcpyDeviceToHost) == hipSuccess ? n : -1;
}
#endif

// one workgroup of a grouped launch: orig = its index among the launch's nwg
// dW workgroups (the XCD-contiguous remap, gemm_tile_index, assumes orig and
// the hardware's blockIdx agree mod 8); gi / rows report the entry and slab
// length for the clock trace
template <int WV>
__device__ __forceinline__ void dwd_group_run(const DwGroup& G, int orig, int nwg, float4* dwd_red,
                                              int& gi, int& rows) {
  int w = orig;
  if (nwg > 8) {                                  // XCD-contiguous runs (gemm_tile_index)
    const int x = orig & 7, q = nwg >> 3, r = nwg & 7;
    w = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (orig >> 3);
  }
  gi = 0;
  while (gi + 1 < G.n && w >= G.wg0[gi + 1]) ++gi;
  const GemmArgs& g = G.g[gi];
  if (g.skip && g.skip[0] != 0) return;
  const int local = w - G.wg0[gi], gn = G.gn[gi], gm = G.gm[gi];
  TileIdx ti;
  ti.nt = local % gn;
  ti.mt = (local / gn) % gm;
  ti.z = local / (gn * gm);
  rows = (min(g.K, (ti.z + 1) * g.kchunk) - ti.z * g.kchunk) |
         ((G.narrow[gi] && ti.mt == gm - 1) << 16) | (G.vec[gi] << 17);
  if (G.narrow[gi] && ti.mt == gm - 1) {
    // a tail of <= 16 gradient rows (M 8 / 200 / 400 at C3) on one 16-wide
    // m sub-tile instead of a 64-wide tile that is >= 75 % padding
    ti.mt *= 4;                                   // m0 = 16 * mt = 64 * (gm - 1)
    if (G.vec[gi] & 1) dwd_tile<1, DWG_NT, false, true, WV>(g, ti, dwd_red);
    else dwd_tile<1, DWG_NT, false, false, WV>(g, ti, dwd_red);
    return;
  }
  switch (G.vec[gi]) {
    case 3: dwd_tile<4, DWG_NT, true, true, WV>(g, ti, dwd_red); break;
    case 2: dwd_tile<4, DWG_NT, true, false, WV>(g, ti, dwd_red); break;
    case 1: dwd_tile<4, DWG_NT, false, true, WV>(g, ti, dwd_red); break;
    default: dwd_tile<4, DWG_NT, false, false, WV>(g, ti, dwd_red); break;
  }
}

template <int WV>
__global__ void __launch_bounds__(64 * WV, WV == 4 ? SMI_DWG_OCC : 1)
gemm_dwd_group_kernel(DwGroup G) {
  extern __shared__ float4 dwd_red[];
  int gi = 0, rows = 0;
#if SMI_DWD_TRACE
  const unsigned long long t_start = wall_clock64(), c_start = clock64();
#endif
  dwd_group_run<WV>(G, blockIdx.x, gridDim.x, dwd_red, gi, rows);
#if SMI_DWD_TRACE
  __syncthreads();
  if (threadIdx.x == 0 && blockIdx.x < kDwTraceMax) {
    g_dw_trace[blockIdx.x][0] = t_start;
    g_dw_trace[blockIdx.x][1] = wall_clock64();
    g_dw_trace[blockIdx.x][2] = __builtin_amdgcn_s_getreg((31 << 11) | 4);
    g_dw_trace[blockIdx.x][3] = __builtin_amdgcn_s_getreg((31 << 11) | 20) | (gi << 8) |
                                ((unsigned long long)rows << 16);
    g_dw_trace[blockIdx.x][4] = c_start;
    g_dw_trace[blockIdx.x][5] = clock64();
  }
#else
  (void)gi; (void)rows;
#endif
}

// BPTT of the one-segment-per-workgroup VALU form (workgroups < la.B) and
// the weight gradients already queued in the phase's group (the heads'; the
// others) in ONE launch: the heads' gradients need nothing from the BPTT, so
// they run on the CUs the recurrence leaves idle (la.B segments on one CU
// each) instead of after it
template <int BR, bool STG>
__global__ void __launch_bounds__(kVT, 1)
lstm_bwd_dw_kernel(LstmBwdArgs la, DwGroup G) {
  extern __shared__ float4 dwd_red[];             // (the BPTT workgroups: their staged step inputs)
  if ((int)blockIdx.x < la.B) {
    lstm_bwd_q_body<BR, SMI_BPTT_CH4 != 0, STG>(la, blockIdx.x, reinterpret_cast<float*>(dwd_red));
    return;
  }
  int gi = 0, rows = 0;
  dwd_group_run<8>(G, blockIdx.x - la.B, gridDim.x - la.B, dwd_red, gi, rows);
}

// the partials of every GEMM of a group, each element summed over its slabs in
// the fixed order of gemm_splitk_reduce_kernel.  With an epilogue task
// (G.x.on): every block also writes the fp64 sum of squares of the values it
// stored to x.sq[block] (fixed order: lane values, wave butterfly, waves in
// order), and one more block (block 0) runs the task itself: the log_var
// gradient from its row partials, that block's sum of squares, the partial
// count and the optimizer step bump (what sumsq_part_kernel and
// logvar_grad_kernel did as launches of their own)
__device__ void dw_epilogue_block(const DwEpilogue& x, int nsq) {
  __shared__ double red[kWG / 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float q = 0.f;
  if (x.lvpart) {
    // d log_var[j] = std_j * sum_blocks lvpart[.][j] (logvar_grad_kernel's order);
    // a wave takes its columns j = wave + 4 i two at a time (both columns'
    // partials in flight together: 16 of the lane's partials per column per
    // trip, the same additions in the same order per column)
    constexpr int NW = kWG / 64;
    for (int j0 = wave; j0 < x.lv_A; j0 += 2 * NW) {
      const int jj[2] = {j0, min(j0 + NW, x.lv_A - 1)};      // (a clamped second column is dropped)
      float t[2] = {0.f, 0.f};
      int i = lane;
      for (; i + 15 * 64 < x.lv_nb; i += 16 * 64) {
        float v[2][16];
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
          for (int k = 0; k < 16; ++k) v[c][k] = x.lvpart[(int64_t)(i + 64 * k) * x.lv_A + jj[c]];
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
          for (int k = 0; k < 16; ++k) t[c] += v[c][k];
      }
      {
        // the tail's loads unconditional (past the end: a zero by address) and
        // pinned before the conditional adds: a load whose only use sat under
        // its lane condition was sunk into that branch, one round trip each
        float v[2][16];
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
          for (int k = 0; k < 16; ++k) {
            const int ik = i + 64 * k;
            v[c][k] = *(ik < x.lv_nb ? x.lvpart + (int64_t)ik * x.lv_A + jj[c] : g_dwd_zero);
          }
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
          for (int k = 0; k < 16; ++k) asm volatile("" : "+v"(v[c][k]));
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
          for (int k = 0; k < 16; ++k)
            if (i + 64 * k < x.lv_nb) t[c] += v[c][k];
      }
      const float e0 = expf(x.lv[jj[0]]), e1 = expf(x.lv[jj[1]]);
      const float g0 = wave_sum(t[0]) * e0;
      const float g1 = wave_sum(t[1]) * e1;
      if (lane == 0) {
        x.lv_out[jj[0]] = g0;
        q += g0 * g0;
        if (j0 + NW < x.lv_A) {
          x.lv_out[jj[1]] = g1;
          q += g1 * g1;
        }
      }
    }
  }
  if (!x.sq) {
    if (threadIdx.x == 0 && x.step) x.step[0] += 1;
    if (threadIdx.x == 0 && x.runs) x.runs[0] += 1;
    return;
  }
  const double t = block_sum_d((double)q, red);
  if (threadIdx.x == 0) {
    x.sq[nsq] = t;
    x.np[0] = nsq + 1;
    if (x.step) x.step[0] += 1;
    if (x.runs) x.runs[0] += 1;
  }
}

// one element's sum over its S slabs as lane zl of the reducer sees it: slabs
// z = zl, zl + 4, ... into four accumulators (z, z + 4, z + 8, z + 12 of each
// 16-slab trip), the rest into the first; p = the element's slab-0 address.
// For S <= 64 every slab is loaded before the first add (one memory round trip):
// the loads are unconditional (slabs past S read a zero by address) and pinned
// before the conditional adds -- with `zk < S ? load : 0` the compiler sank
// each load into its own branch and waited on it there, and 64-bit index
// products per load made it reuse address registers between loads (round 6)
template <int U>
__device__ __forceinline__ void red_slabs(const float* const (&p)[U], int64_t MN, int S, int zl,
                                          float (&r)[U]) {
  float s0[U], s1[U], s2[U], s3[U];
#pragma unroll
  for (int u = 0; u < U; ++u) s0[u] = s1[u] = s2[u] = s3[u] = 0.f;
  int z = zl;
  if (S <= 64) {
    const int64_t st4 = 4 * MN;
    float v[U][16];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const float* pz = p[u] + (int64_t)zl * MN;
#pragma unroll
      for (int k = 0; k < 16; ++k) v[u][k] = *(zl + 4 * k < S ? pz + k * st4 : g_dwd_zero);
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int k = 0; k < 16; ++k) asm volatile("" : "+v"(v[u][k]));
    const int nfull = S > zl + 12 ? (S - zl - 12 + 15) / 16 : 0;   // z + 12 < S trips
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (j < nfull) {
          s0[u] += v[u][4 * j]; s1[u] += v[u][4 * j + 1]; s2[u] += v[u][4 * j + 2]; s3[u] += v[u][4 * j + 3];
        }
      }
#pragma unroll
      for (int k = 0; k < 16; ++k)
        if (k >= 4 * nfull && zl + 4 * k < S) s0[u] += v[u][k];
    }
    z = S;
  }
  for (; z + 12 < S; z += 16) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      s0[u] += p[u][(int64_t)z * MN];
      s1[u] += p[u][(int64_t)(z + 4) * MN];
      s2[u] += p[u][(int64_t)(z + 8) * MN];
      s3[u] += p[u][(int64_t)(z + 12) * MN];
    }
  }
  for (; z < S; z += 4)
#pragma unroll
    for (int u = 0; u < U; ++u) s0[u] += p[u][(int64_t)z * MN];
#pragma unroll
  for (int u = 0; u < U; ++u) r[u] = (s0[u] + s1[u]) + (s2[u] + s3[u]);
}

// U: 64-element groups per block (block = 64 U consecutive elements; lane el
// of wave zl sums slabs zl, zl + 4, ... of elements el + 64 u).  Every element
// gets the additions of gemm_splitk_reduce_kernel in the same order whatever
// U is; U = 4 dispatches a quarter of the workgroups with 4x the loads in
// flight per thread (SMI_RED_U, host side)
template <int U>
__global__ void __launch_bounds__(kWG)
gemm_group_reduce_kernel(DwGroup G) {
  __shared__ float red[4][64 * U];
  __shared__ double sqr[kWG / 64];
  // the epilogue task (when on) is block 0: dispatched first, its chain of
  // dependent steps overlaps the reduction blocks instead of trailing them
  const int ep = G.x.on ? 1 : 0;
  if (ep && blockIdx.x == 0) {
    if (G.x.skip && G.x.skip[0] != 0) return;
    dw_epilogue_block(G.x, G.rb0[G.n]);
    return;
  }
  const int b = (int)blockIdx.x - ep;
  int gi = 0;
  while (gi + 1 < G.n && b >= G.rb0[gi + 1]) ++gi;
  const GemmArgs& g = G.g[gi];
  if (g.skip && g.skip[0] != 0) return;
  const int S = G.S[gi];
  const int64_t MN = (int64_t)g.M * g.N;
  const int el = threadIdx.x & 63, zl = threadIdx.x >> 6;
  const int64_t eb = (int64_t)(b - G.rb0[gi]) * 64 * U;
  const float* p[U];
#pragma unroll
  for (int u = 0; u < U; ++u) p[u] = g.part + min(eb + el + 64 * u, MN - 1);
  float r[U];
  red_slabs<U>(p, MN, S, zl, r);
#pragma unroll
  for (int u = 0; u < U; ++u) red[zl][el + 64 * u] = r[u];
  __syncthreads();
  float q = 0.f;
  for (int i = threadIdx.x; i < 64 * U; i += kWG) {
    const int64_t e = eb + i;
    if (e < MN) {
      const float v = (red[0][i] + red[1][i]) + (red[2][i] + red[3][i]);
      const int m = (int)(e / g.N), n = (int)(e - (int64_t)m * g.N);
      q += dw_put(g, m, n, v);
    }
  }
  if (!G.x.sq) return;
  const double t = block_sum_d((double)q, sqr);
  if (threadIdx.x == 0) G.x.sq[b] = t;
}


// Row-panel GEMM for the learner's tall activations (rows >> N, K small):
//   EPI_FWD: Y = act(X W^T + b)        EPI_DX: dX = (dY W) * [mask > 0]
// A workgroup owns 64 rows x 16*NTW output columns, one 16-row MFMA tile per
// wave.  The A operand goes from global memory straight into MFMA registers
// as 16-byte k-runs (lane (li, lk) loads row li, k 4lk..4lk+3 of a 16-k
// chunk; B is staged with the same k permutation), so every activation row
// is read once per column group; the weight chunk B[16 k][16*NTW n] is
// staged in LDS once per workgroup and shared by the four waves (one barrier
// per chunk).  k past K reads a zero row by address (g_dwd_zero).
constexpr int PN_LD = 20;

template <int EPI, int NTW>
__global__ void __launch_bounds__(kWG)
gemm_panel_kernel(GemmArgs g) {
  if (g.skip && g.skip[0] != 0) return;
  constexpr int NB = 16 * NTW;                    // columns per workgroup
  constexpr int BQ = (4 * NB + kWG - 1) / kWG;    // staged float4 per thread
  __shared__ __attribute__((aligned(16))) float sB[2][NB * PN_LD + 4];   // + dummy slot
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, lk = lane >> 4;
  const TileIdx ti = gemm_tile_index();
  const int r0 = ti.mt * 64 + wave * 16;
  const int n0 = ti.nt * NB;
  const int nch = (g.K + 15) >> 4;
  const float* arow = g.A + (int64_t)min(r0 + li, g.M - 1) * g.a_rs;
  auto load_a = [&](int c) -> float4 {
    const int k = c * 16 + 4 * lk;
    return *reinterpret_cast<const float4*>(k < g.K ? arow + k : g_dwd_zero);
  };
  // staging: FWD B(k, n) = W[n][k] (k-contiguous rows); DX B(k, n) = W[k][n].
  // Slot q of this thread is element idx = tid + q*256 of the chunk; slots past
  // the chunk (idx >= 4*NB) load the zero row and write the dummy LDS slot (no
  // divergent branches: the staging values stay in named registers)
  auto load_b = [&](int c, int q) -> float4 {
    const int idx = tid + q * kWG;
    const float* src;
    if constexpr (EPI == EPI_FWD) {
      const int n = idx >> 2, k = c * 16 + ((idx & 3) << 2);
      const int nc = min(n0 + n, g.N - 1);
      src = (idx < 4 * NB && k < g.K) ? g.B + (int64_t)nc * g.b_cs + k : g_dwd_zero;
    } else {
      const int k = idx / (NB / 4), nq = (idx - k * (NB / 4)) << 2;
      const int kk = c * 16 + k;
      const int nc = min(n0 + nq, g.N - 4);
      src = (idx < 4 * NB && kk < g.K) ? g.B + (int64_t)kk * g.b_rs + nc : g_dwd_zero;
    }
    return *reinterpret_cast<const float4*>(src);
  };
  auto store_b = [&](float* S, int q, float4 r) {
    const int idx = tid + q * kWG;
    const bool ok = idx < 4 * NB;
    if constexpr (EPI == EPI_FWD) {
      const int n = idx >> 2, kq = (idx & 3) << 2;
      *reinterpret_cast<float4*>(S + (ok ? n * PN_LD + kq : NB * PN_LD)) = r;
    } else {
      const int k = idx / (NB / 4), nq = (idx - k * (NB / 4)) << 2;
      const int base = ok ? nq * PN_LD + k : NB * PN_LD;
      const int step = ok ? PN_LD : 1;
      S[base] = r.x; S[base + step] = r.y; S[base + 2 * step] = r.z; S[base + 3 * step] = r.w;
    }
  };
  f32x4 acc[NTW];
#pragma unroll
  for (int b = 0; b < NTW; ++b) acc[b] = f32x4{0.f, 0.f, 0.f, 0.f};
  static_assert(BQ <= 3, "panel staging: at most 3 float4 per thread");
  float4 b0, b1, b2;
  float4 aC = load_a(0), aN;
  b0 = load_b(0, 0);
  if constexpr (BQ > 1) b1 = load_b(0, 1);
  if constexpr (BQ > 2) b2 = load_b(0, 2);
  store_b(sB[0], 0, b0);
  if constexpr (BQ > 1) store_b(sB[0], 1, b1);
  if constexpr (BQ > 2) store_b(sB[0], 2, b2);
  __syncthreads();
  for (int c = 0; c < nch; ++c) {
    const bool more = c + 1 < nch;
    if (more) {
      aN = load_a(c + 1);
      b0 = load_b(c + 1, 0);
      if constexpr (BQ > 1) b1 = load_b(c + 1, 1);
      if constexpr (BQ > 2) b2 = load_b(c + 1, 2);
    }
    const float* S = sB[c & 1];
    float4 bq[NTW];
#pragma unroll
    for (int b = 0; b < NTW; ++b)
      bq[b] = *reinterpret_cast<const float4*>(S + (16 * b + li) * PN_LD + 4 * lk);
#pragma unroll
    for (int b = 0; b < NTW; ++b) {
      acc[b] = mfma4(aC.x, bq[b].x, acc[b]);
      acc[b] = mfma4(aC.y, bq[b].y, acc[b]);
      acc[b] = mfma4(aC.z, bq[b].z, acc[b]);
      acc[b] = mfma4(aC.w, bq[b].w, acc[b]);
    }
    if (more) {
      float* S1 = sB[(c + 1) & 1];
      store_b(S1, 0, b0);
      if constexpr (BQ > 1) store_b(S1, 1, b1);
      if constexpr (BQ > 2) store_b(S1, 2, b2);
      aC = aN;
    }
    __syncthreads();
  }
#pragma unroll
  for (int b = 0; b < NTW; ++b) {
    const int n = n0 + 16 * b + li;
    if (n >= g.N) continue;
    float bias_n = 0.f;
    if constexpr (EPI == EPI_FWD) bias_n = g.bias ? g.bias[n] : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = r0 + 4 * lk + i;
      if (m >= g.M) continue;
      float v = acc[b][i];
      if constexpr (EPI == EPI_FWD) {
        v += bias_n;
        if (g.act == ACT_RELU) v = v > 0.f ? v : 0.f;
        else if (g.act == ACT_TANH) v = tanhf(v);
      } else {
        if (g.mask) v = g.mask[(int64_t)m * g.ldm + n] > 0.f ? v : 0.f;
      }
      g.C[(int64_t)m * g.ldc + n] = v;
    }
  }
}

float* workspace_f32(int64_t nfloats);

// split-K target workgroup count (SMI_SPLITK_TARGET overrides; tuning knob)
static int smi_splitk_target() {
  static int t = 0;
  if (!t) {
    const char* e = getenv("SMI_SPLITK_TARGET");
    t = e ? atoi(e) : 512;
    if (t < 64) t = 64;
  }
  return t;
}

template <int EPI>
static void gemm_dispatch(const GemmArgs& g, dim3 grid, bool ak, bool bk, hipStream_t st) {
  if (ak && bk) hipLaunchKernelGGL((gemm_kernel<EPI, true, true>), grid, dim3(kWG), 0, st, g);
  else if (ak) hipLaunchKernelGGL((gemm_kernel<EPI, true, false>), grid, dim3(kWG), 0, st, g);
  else if (bk) hipLaunchKernelGGL((gemm_kernel<EPI, false, true>), grid, dim3(kWG), 0, st, g);
  else hipLaunchKernelGGL((gemm_kernel<EPI, false, false>), grid, dim3(kWG), 0, st, g);
}

static int use_dwd() {
  static int u = -1;
  if (u < 0) {
    const char* e = getenv("SMI_DWD");
    u = (e && e[0] == '0') ? 0 : 1;
  }
  return u;
}

template <int MT, int NT, int WV>
static void dwd_dispatch(const GemmArgs& g, dim3 grid, bool va, bool vb, hipStream_t st) {
  const size_t lds = (size_t)2 * MT * NT * 64 * sizeof(float4);
  const dim3 blk(64 * WV);
  if (va && vb) hipLaunchKernelGGL((gemm_dwd_kernel<MT, NT, true, true, WV>), grid, blk, lds, st, g);
  else if (va) hipLaunchKernelGGL((gemm_dwd_kernel<MT, NT, true, false, WV>), grid, blk, lds, st, g);
  else if (vb) hipLaunchKernelGGL((gemm_dwd_kernel<MT, NT, false, true, WV>), grid, blk, lds, st, g);
  else hipLaunchKernelGGL((gemm_dwd_kernel<MT, NT, false, false, WV>), grid, blk, lds, st, g);
}

// waves per dW workgroup (SMI_DWD_WAVES=4|8; measured: 8 waves, two per
// SIMD, 5-10 % slower per launch and 6 % slower end to end at C3)
static int dwd_waves() {
  static int w = 0;
  if (!w) {
    const char* e = getenv("SMI_DWD_WAVES");
    w = (e && atoi(e) == 8) ? 8 : 4;
  }
  return w;
}

static int splitk_reduce(const GemmArgs& g, int S, int epi, hipStream_t st);

// weight gradient over row-major dY / X (a_rs == 1, b_cs == 1): gemm_dwd_kernel
static int dwd_launch(GemmArgs g, hipStream_t st) {
  auto al16 = [](const float* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  const int bdata = g.ones_col >= 0 ? g.ones_col : g.N;
  const int MT = g.M > 32 ? 4 : 1, NT = g.N > 64 ? 8 : 4;
  const bool va = MT == 4 && al16(g.A) && g.M % 4 == 0 && g.a_cs % 4 == 0;
  const bool vb = al16(g.B) && bdata >= 4 && bdata % 4 == 0 && g.b_rs % 4 == 0 &&
                  (!g.B2 || (al16(g.B2) && g.b2_rs % 4 == 0 && g.split_col % 4 == 0));
  const int gm = (g.M + 16 * MT - 1) / (16 * MT), gn = (g.N + 16 * NT - 1) / (16 * NT);
  const int tiles = gm * gn;
  static int target = 0;
  if (!target) {    // measured: ~1 workgroup per CU beats deeper splits (partials)
    const char* e = getenv("SMI_DWD_TARGET");
    target = e ? atoi(e) : 256;
    if (target < 16) target = 16;
  }
  int S = (target + tiles - 1) / tiles;
  const int smax = (g.K + 32 * dwd_waves() - 1) / (32 * dwd_waves());   // >= 8 steps per wave
  if (S > smax) S = smax;
  const int64_t cap = smi_workspace_floats() / ((int64_t)g.M * g.N);
  if (S > cap) S = (int)cap;
  if (S < 1) S = 1;
  g.part = nullptr;
  g.kchunk = g.K;
  if (S > 1) {
    const int rs = 4 * dwd_waves() * DWD_P;        // rows per prefetch window
    g.kchunk = ((g.K + S - 1) / S + rs - 1) / rs * rs;
    S = (g.K + g.kchunk - 1) / g.kchunk;
  }
  if (S > 1) {
    g.part = workspace_f32((int64_t)S * g.M * g.N);
    if (!g.part) return set_error(SMI_E_ARG, "gemm: workspace unavailable for split-K");
  }
  const dim3 grid(gm, gn, S);
  const int kslot = ktime_begin(st);
  if (dwd_waves() == 8) {
    if (MT == 4 && NT == 8) dwd_dispatch<4, 8, 8>(g, grid, va, vb, st);
    else if (MT == 4) dwd_dispatch<4, 4, 8>(g, grid, va, vb, st);
    else if (NT == 8) dwd_dispatch<1, 8, 8>(g, grid, false, vb, st);
    else dwd_dispatch<1, 4, 8>(g, grid, false, vb, st);
  } else {
    if (MT == 4 && NT == 8) dwd_dispatch<4, 8, 4>(g, grid, va, vb, st);
    else if (MT == 4) dwd_dispatch<4, 4, 4>(g, grid, va, vb, st);
    else if (NT == 8) dwd_dispatch<1, 8, 4>(g, grid, false, vb, st);
    else dwd_dispatch<1, 4, 4>(g, grid, false, vb, st);
  }
  const int nreal = (g.ones_col >= 0 ? g.N - 1 : g.N) -
                    (g.B2 ? g.split_col - g.c1_real : 0);      // padding columns do no work
  ktime_end(kslot, KT_GEMM_DW,
            2.0 * g.M * (double)nreal * g.K + (g.ones_col >= 0 ? (double)g.M * g.K : 0.0), st);
  const int rc = check_launch("gemm_dwd_kernel");
  if (rc || S == 1) return rc;
  return splitk_reduce(g, S, EPI_DW, st);
}

// ---- grouped weight gradients (gemm_dwd_group_kernel) ----------------------
// whether an M x N weight gradient over row-major operands joins an open group
// (gemm_launch's rule; the dW2 / bias column included in N by the caller)
bool dw_group_takes(int M, int N) { return use_dwd() && M >= 1 && N >= 1 && M <= 512 && N <= 512; }

// the queue of the calling thread (begin ... flush bracket one call sequence)
static thread_local DwGroup g_grp;
static thread_local bool g_grp_on = false;
static thread_local double g_grp_flops = 0.0;
// set when a weight gradient issued inside an open bracket did not join the
// group (group full, or a shape / layout the grouped kernel does not take):
// with a fused sum of squares (x.sq) its gradient would be missing from the
// clip_grad_norm_ partials, so the flush fails instead of clipping wrongly
static thread_local bool g_grp_missed = false;

int dw_group_begin() {
  g_grp_on = true;
  g_grp_missed = false;
  g_grp.n = 0;
  g_grp.x = DwEpilogue{};
  g_grp_flops = 0.0;
  return SMI_OK;
}

// the reducer's epilogue task of the open group (dw_group_flush launches one
// more reducer block for it); with x.sq every weight gradient of the bracket
// must join the group (the fused sum of squares covers only the group)
int dw_group_epilogue(const DwEpilogue& x) {
  if (!g_grp_on) return set_error(SMI_E_ARG, "dw group: no open group for the epilogue");
  g_grp.x = x;
  g_grp.x.on = 1;
  return SMI_OK;
}

static bool dw_group_add(const GemmArgs& g) {
  if (!g_grp_on) return false;
  if (g_grp.n >= kDwGroupMax) {
    g_grp_missed = true;
    return false;
  }
  auto al16 = [](const float* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  const int bdata = g.ones_col >= 0 ? g.ones_col : g.N;
  const bool va = al16(g.A) && g.M >= 4 && g.M % 4 == 0 && g.a_cs % 4 == 0;
  const bool vb = al16(g.B) && bdata >= 4 && bdata % 4 == 0 && g.b_rs % 4 == 0 &&
                  (!g.B2 || (al16(g.B2) && g.b2_rs % 4 == 0 && g.split_col % 4 == 0));
  const int i = g_grp.n++;
  g_grp.g[i] = g;
  g_grp.vec[i] = (va ? 2 : 0) + (vb ? 1 : 0);
  const int nreal = (g.ones_col >= 0 ? g.N - 1 : g.N) - (g.B2 ? g.split_col - g.c1_real : 0);
  g_grp_flops += 2.0 * g.M * (double)nreal * g.K + (g.ones_col >= 0 ? (double)g.M * g.K : 0.0);
  return true;
}

// target workgroups of a grouped launch for `work` tile-rows (SMI_DWD_GROUP_TARGET
// overrides; tuning knob).  Measured at C3 (bench, one MI355X), 21504 rows:
// 256 -> 4.44 ms of dW per learn, 512 -> 3.71, 768 -> 3.17, 1024 -> 2.83
// (45 TF/s), 1536 -> 3.32, 3072 -> 4.43; at 2688 rows (one rank of eight,
// tools/bench_dwgroup.py --segments 128): 1024 -> 65 us per launch (128-row
// slabs), 512 -> 48, 256 -> 46: slabs shorter than ~384 rows are all ramp.
// With the 64 x 64 tiles at 3 waves per SIMD (DWG_NT below): 1024 -> 120.5 us
// per C3 launch, 1536 -> 110.0 (0.37 of the f32 MFMA peak), 2048 -> 110.5.
// Round 5, 128 segments (3200 rows): the LSTM's gradient alone (the heads'
// run with the BPTT) at 128 / 175 (work / 384) / 256 / 384 workgroups: 23.8 /
// 22.9 / 21.1 / 21.3 us; the whole group at 512 vs 458: 26.5 vs 28.0 us —
// work / 256.
static int dw_group_target(double work) {
  static int t = -1;
  if (t < 0) {
    const char* e = getenv("SMI_DWD_GROUP_TARGET");
    t = (e && e[0]) ? atoi(e) : 0;
    if (e && e[0] && t < 64) t = 64;
  }
  if (t > 0) return t;
  const double w = work / 256.0;
  return w >= 1536.0 ? 1536 : w <= 128.0 ? 128 : (int)w;
}

// narrow 16-wide tail tiles in grouped launches (SMI_DWD_NARROW=0: off; A/B knob)
static int use_dwd_narrow() {
  static int u = -1;
  if (u < 0) {
    const char* e = getenv("SMI_DWD_NARROW");
    u = (e && e[0] == '0') ? 0 : 1;
  }
  return u;
}

// relative time per row of a 16-wide tail tile against a full 64 x 64 tile
// (per-workgroup clock trace of the C3 launch, tools/bench_dwgroup.py with the
// `dwtrace` build: 832-row slabs took 18.3 us on tail tiles, 47 us on full ones)
static double dwd_narrow_cost() {
  static double c = -1.0;
  if (c < 0.0) {
    const char* e = getenv("SMI_DWD_NARROW_COST");
    c = (e && e[0]) ? atof(e) : 0.4;
    if (c <= 0.0 || c > 1.0) c = 0.4;
  }
  return c;
}

// Workgroups of one grouped launch resident at once (CUs x occupancy).
static int dwd_group_slots(size_t lds) {
  static int slots = 0;
  if (!slots) {
    slots = dwd_waves() == 8 ? resident_grid(gemm_dwd_group_kernel<8>, 512, lds)
                             : resident_grid(gemm_dwd_group_kernel<4>, 256, lds);
    if (slots < 1) slots = 256;
  }
  return slots;
}

// Tail splits, balanced slabs and the split-K partials of G's entries, placed
// ws_off floats into the workspace; wv: waves per workgroup of the launch that
// runs them, slots: its resident workgroups.  Sets G.wg0 / rb0 / S / part and
// need (floats used from ws_off).
// 64-element groups per block of the grouped reducer (SMI_RED_U=1: one, the
// round-5 form; A/B knob)
static int red_u() {
  static const int u = [] { const char* e = getenv("SMI_RED_U"); return e && e[0] == '1' ? 1 : 4; }();
  return u;
}

static int dw_prepare(DwGroup& G, int wv, int slots, int64_t ws_off, int64_t& need,
                      int target_fixed = 0) {
  constexpr int MT = 4, NT = DWG_NT;
  const int rs = 4 * wv * DWD_P;                    // rows per prefetch window
  auto al16 = [](const float* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  // A GEMM whose last m-tile is a <= 16-row tail (M 8 / 200 / 400 at C3) is
  // split, while the group has room, into its full 64-row tiles and a tail
  // entry: the tail's tiles then get their own, longer slabs (below).  The
  // tail entry addresses rows m0.. of dY and of every destination.
  {
    const int n0 = G.n;
    DwGroup E = G;
    int n = 0;
    for (int i = 0; i < n0; ++i) {
      const GemmArgs& g = G.g[i];
      const int tail = g.M % (16 * MT);
      const bool split = use_dwd_narrow() && tail > 0 && tail <= 16 && g.M > 16 * MT &&
                         g.a_rs == 1 && n + (n0 - i) + 1 <= kDwSplitMax;
      E.g[n] = g;
      E.vec[n] = G.vec[i];
      if (!split) { ++n; continue; }
      const int m0 = g.M - tail;
      E.g[n].M = m0;                                  // the full tiles (vec unchanged)
      ++n;
      GemmArgs t = g;
      t.M = tail;
      t.A = g.A + m0;
      if (t.C) t.C = g.C + (int64_t)m0 * g.ldc;
      if (t.C2) t.C2 = g.C2 + (int64_t)m0 * g.ldc2;
      if (t.bias_out) t.bias_out = g.bias_out + m0;
      if (t.bias_out2) t.bias_out2 = g.bias_out2 + m0;
      const bool va = al16(t.A) && t.M >= 4 && t.M % 4 == 0 && t.a_cs % 4 == 0;
      E.g[n] = t;
      E.vec[n] = (va ? 2 : 0) + (G.vec[i] & 1);
      ++n;
    }
    E.n = n;
    G = E;
  }
  // Balanced workgroups.  A launch with more work than one resident round
  // (CUs x occupancy) runs as whole rounds (one at C3: a second, partly filled
  // round was the launch's tail — the per-workgroup clock trace showed the
  // last 40 % of the span at falling concurrency), and each entry's slab
  // length is set so that its slabs cost about the same time (tail tiles ~0.4
  // of a full tile per row).  Below one round every workgroup is resident
  // anyway and the span is the longest slab: equal slab lengths (shorter
  // fp32 chains on the tail tiles).
  double cost[kDwGroupMax], work = 0.0, work_u = 0.0;  // tiles x rows (x cost)
  int64_t tiles[kDwGroupMax];
  for (int i = 0; i < G.n; ++i) {
    const GemmArgs& g = G.g[i];
    const int tail = g.M % (16 * MT);
    G.narrow[i] = use_dwd_narrow() && tail > 0 && tail <= 16;
    G.gm[i] = (g.M + 16 * MT - 1) / (16 * MT);
    G.gn[i] = (g.N + 16 * NT - 1) / (16 * NT);
    tiles[i] = (int64_t)G.gm[i] * G.gn[i];
    cost[i] = G.narrow[i] ? ((G.gm[i] - 1) + dwd_narrow_cost()) / G.gm[i] : 1.0;
    work_u += (double)tiles[i] * g.K;
    work += (double)tiles[i] * g.K * cost[i];
  }
  int target = target_fixed > 0 ? target_fixed : dw_group_target(work_u);
  static const bool env_target = [] {
    const char* e = getenv("SMI_DWD_GROUP_TARGET");
    return e && e[0];
  }();
  const bool fixed_target = env_target || target_fixed > 0;
  if (!fixed_target && target >= slots) {
    // whole rounds of at most ~2048 cost-rows per workgroup (SMI_DWD_ROUND_ROWS)
    static const double round_rows = [] {
      const char* e = getenv("SMI_DWD_ROUND_ROWS");
      const double v = (e && e[0]) ? atof(e) : 2048.0;
      return v >= 256.0 ? v : 2048.0;
    }();
    const int rounds = (int)std::max(1.0, std::ceil(work / (slots * round_rows)));
    target = slots * rounds;
  } else {
    for (int i = 0; i < G.n; ++i) cost[i] = 1.0;
    work = work_u;
  }
  const int64_t cap = smi_workspace_floats() - ws_off;
  double r0 = work / target;                        // cost-rows per workgroup
  int64_t kcs[kDwGroupMax];
  // slab lengths are rounded up to whole prefetch windows, so the workgroup
  // count can land a few above the target; in whole rounds every extra
  // workgroup is a second round of its own (the C3 launch was 769 for 768
  // slots: the last workgroup started at 59 us and set the span), so the
  // cost-rows per workgroup grow in small steps until the count fits
  const bool rounds_fit = !fixed_target && target >= slots;
  need = 0;
  for (int pass = 0; pass < 400; ++pass) {
    need = 0;
    int64_t wgs = 0;
    for (int i = 0; i < G.n; ++i) {
      const GemmArgs& g = G.g[i];
      int64_t S = (int64_t)(g.K * cost[i] / r0 + 0.5);
      if (S < 1) S = 1;
      int64_t kc = ((g.K + S - 1) / S + rs - 1) / rs * rs;
      if (kc < 2 * rs) kc = 2 * rs;                 // >= 8 MFMA steps per wave
      if (kc >= g.K) kc = ((int64_t)g.K + rs - 1) / rs * rs;
      kcs[i] = kc;
      const int64_t s_i = (g.K + kc - 1) / kc;
      need += s_i * g.M * g.N;
      wgs += s_i * tiles[i];
    }
    if (need > cap) { r0 *= 2.0; continue; }         // grow the slabs until the partials fit
    if (rounds_fit && wgs > target && wgs <= 2 * target) { r0 *= 1.005; continue; }
    break;
  }
  float* base = workspace_f32(ws_off + need);
  if (!base) return set_error(SMI_E_ARG, "gemm: workspace too small for the grouped dW partials");
  base += ws_off;
  int64_t off = 0;
  G.wg0[0] = 0;
  G.rb0[0] = 0;
  for (int i = 0; i < G.n; ++i) {
    GemmArgs& g = G.g[i];
    g.kchunk = (int)kcs[i];
    G.S[i] = (int)((g.K + kcs[i] - 1) / kcs[i]);
    g.part = base + off;
    off += (int64_t)G.S[i] * g.M * g.N;
    G.wg0[i + 1] = G.wg0[i] + (int)(tiles[i] * G.S[i]);
    G.rb0[i + 1] = G.rb0[i] + (int)(((int64_t)g.M * g.N + 64 * red_u() - 1) / (64 * red_u()));
  }
  return SMI_OK;
}

// short-batch 16 x 16-tile kernels (gemm_t16_kernel, gemm_dwt16_kernel): 16-k
// chunks per wave, K <= 4 * 16 * 8 = 512
constexpr int T16_MAXC = 8;
// SMI_GEMM_T16=0: the split-K / grouped forms for short batches instead (A/B knob)
static bool use_t16() {
  static const bool on = [] { const char* e = getenv("SMI_GEMM_T16"); return !(e && e[0] == '0'); }();
  return on;
}

// Weight gradients of short batches without split-K: one 16 x 16 tile of one
// group entry per workgroup, the four waves splitting the rows in 16-row
// chunks (wave w takes c = w, w + 4, ...) through a ring of DR chunks in
// flight, two accumulator chains (even / odd chunk of the wave), a fixed-order
// LDS sum of the four waves, then the destination written directly (dw_put:
// no partials, no reducer launch).  Lane (i, q) reads dY[k][m0 + i] and
// X[k][n0 + i] for k = 16c + 4q + s: 16 consecutive floats per row on both
// operands.  The two-source B of the LSTM's [x_t | h_{t-1}] (B2) and the
// bias column are formed per lane.  Measured on the LSTM's gradient at 3200
// rows (a rank's batch): 28-30 us against 21.6 us on the grouped dW launch
// (800 scalar operand loads per lane), so only short groups take it.
constexpr int DWT_DR = 8;   // chunks in flight per wave (the trip's accumulators)
__global__ void __launch_bounds__(kWG)
gemm_dwt16_kernel(DwGroup G) {
  __shared__ f32x4 red[4][64];
  const int b = blockIdx.x;
  int gi = 0;
  while (gi + 1 < G.n && b >= G.wg0[gi + 1]) ++gi;
  const GemmArgs& g = G.g[gi];
  if (g.skip && g.skip[0] != 0) return;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int i = lane & 15, q = lane >> 4;
  const int local = b - G.wg0[gi], gn16 = (g.N + 15) >> 4;
  const int m0 = (local / gn16) * 16, n0 = (local % gn16) * 16;
  const int mi = min(m0 + i, g.M - 1), ni = n0 + i;
  const int bdata = g.ones_col >= 0 ? g.ones_col : g.N;
  const float* Ar = g.A + (int64_t)mi * g.a_rs;
  // column ni of B: the first source, the second (B2: columns >= split_col),
  // a padding column (c1_real <= ni < split_col), the bias column or past N
  const float* Bc = g.B;
  int64_t bs = g.b_rs;
  bool bz = false, bone = false;
  if (ni == g.ones_col) bone = true;
  else if (ni >= bdata || ni >= g.N) bz = true;
  else if (g.B2 && ni >= g.split_col) { Bc = g.B2 + (ni - g.split_col); bs = g.b2_rs; }
  else if (g.B2 && ni >= g.c1_real) bz = true;
  else Bc = g.B + (int64_t)ni * g.b_cs;
  const int nch = (g.K + 15) >> 4;
  const int nw = nch > wave ? (nch - wave + 3) >> 2 : 0;        // this wave's chunks
  float av[DWT_DR][4], bv[DWT_DR][4];
  auto ld = [&](int j, int slot) {
    const int c = wave + 4 * j;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int k = 16 * c + 4 * q + t;
      const bool kv = j < nw && k < g.K;
      av[slot][t] = kv ? Ar[(int64_t)k * g.a_cs] : 0.f;
      bv[slot][t] = kv ? (bone ? 1.f : bz ? 0.f : Bc[(int64_t)k * bs]) : 0.f;
    }
  };
#pragma unroll
  for (int d = 0; d < DWT_DR; ++d) ld(d, d);
  // each ring trip: one fresh MFMA chain per slot (16 products), the trip's
  // four chains summed in a fixed tree into the running total (short fp32
  // chains: at 3200 rows a single chain per wave was ~2x the oracle's fp32
  // spread on the C3 rank fixture's update bars)
  f32x4 tot = {0.f, 0.f, 0.f, 0.f};
  for (int j0 = 0; j0 < nw; j0 += DWT_DR) {
    f32x4 acc[DWT_DR];
#pragma unroll
    for (int d = 0; d < DWT_DR; ++d) {
      acc[d] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (j0 + d < nw) {
#pragma unroll
        for (int t = 0; t < 4; ++t) acc[d] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[d][t], bv[d][t], acc[d], 0, 0, 0);
      }
      ld(j0 + d + DWT_DR, d);
    }
    tot += ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
  }
  red[wave][lane] = tot;
  __syncthreads();
  if (wave != 0) return;
  const f32x4 sum = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
  if (ni >= g.N) return;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int m = m0 + 4 * q + r;
    if (m < g.M) dw_put(g, m, ni, sum[r]);
  }
}

static void dwt16_prefix(DwGroup& G) {
  G.wg0[0] = 0;
  for (int i = 0; i < G.n; ++i)
    G.wg0[i + 1] = G.wg0[i] + ((G.g[i].M + 15) / 16) * ((G.g[i].N + 15) / 16);
}

// entries already launched with the BPTT (launch_lstm_bwd_dw) whose partials
// the group's reducer still sums, and the workspace floats they hold
static thread_local DwGroup g_pre;
static thread_local bool g_pre_on = false;
static thread_local int64_t g_pre_need = 0;

constexpr size_t kDwdLds = (size_t)2 * 4 * DWG_NT * 64 * sizeof(float4);

int dw_group_flush(hipStream_t st) {
  g_grp_on = false;
  DwGroup& G = g_grp;
  const bool missed = g_grp_missed;
  g_grp_missed = false;
  const bool pre = g_pre_on;
  g_pre_on = false;
  // the pre partials stay reserved through this flush's own requests (its
  // partials land above them), released on every return
  struct Release { ~Release() { workspace_reserve(0); } } release_;
  if (G.x.on && G.x.sq && missed)
    return set_error(SMI_E_ARG, "dw group: a fused sum of squares needs every dW GEMM of the "
                                "bracket in the group (one ran outside it)");
  if (G.n == 0 && !pre) {
    if (!G.x.on) return SMI_OK;
    if (G.x.sq) return set_error(SMI_E_ARG, "dw group: fused sum of squares over an empty group");
    G.rb0[0] = 0;                                   // the epilogue task alone
    hipLaunchKernelGGL(gemm_group_reduce_kernel<1>, dim3(1), dim3(kWG), 0, st, G);
    return check_launch("gemm_group_reduce_kernel");
  }
  // short batches (every entry <= 512 rows, one group, no epilogue task):
  // 16 x 16 tiles written directly, no partials and no reducer
  if (!pre && !G.x.on && use_t16()) {
    bool small = G.n > 0;
    for (int i = 0; i < G.n; ++i) small = small && G.g[i].K <= 4 * 16 * T16_MAXC;
    if (small) {
      dwt16_prefix(G);
      const int kslot = ktime_begin(st);
      hipLaunchKernelGGL(gemm_dwt16_kernel, dim3(G.wg0[G.n]), dim3(kWG), 0, st, G);
      ktime_end(kslot, KT_GEMM_DW, g_grp_flops, st);
      return check_launch("gemm_dwt16_kernel");
    }
  }
  int64_t need = 0;
  if (G.n > 0) {
    RC_CHECK(dw_prepare(G, dwd_waves(), dwd_group_slots(kDwdLds), 0, need));
    const int kslot = ktime_begin(st);
    if (dwd_waves() == 8)
      hipLaunchKernelGGL(gemm_dwd_group_kernel<8>, dim3(G.wg0[G.n]), dim3(512), kDwdLds, st, G);
    else
      hipLaunchKernelGGL(gemm_dwd_group_kernel<4>, dim3(G.wg0[G.n]), dim3(256), kDwdLds, st, G);
    ktime_end(kslot, KT_GEMM_DW, g_grp_flops, st);
    RC_CHECK(check_launch("gemm_dwd_group_kernel"));
  }
  // the reducer sums the partials of the entries launched with the BPTT and
  // of these, in one launch
  DwGroup R = G;
  if (pre) {
    R = g_pre;
    R.x = G.x;
    if (R.n + G.n > kDwGroupMax) return set_error(SMI_E_ARG, "dw group: too many entries");
    for (int i = 0; i < G.n; ++i) {
      const int j = R.n + i;
      R.g[j] = G.g[i];
      R.S[j] = G.S[i];
      R.rb0[j + 1] = R.rb0[j] + (int)(((int64_t)G.g[i].M * G.g[i].N + 64 * red_u() - 1) / (64 * red_u()));
    }
    R.n += G.n;
    need += g_pre_need;
  }
  const int rslot = ktime_begin(st);
  if (red_u() == 4)
    hipLaunchKernelGGL(gemm_group_reduce_kernel<4>, dim3(R.rb0[R.n] + (R.x.on ? 1 : 0)), dim3(kWG), 0,
                       st, R);
  else
    hipLaunchKernelGGL(gemm_group_reduce_kernel<1>, dim3(R.rb0[R.n] + (R.x.on ? 1 : 0)), dim3(kWG), 0,
                       st, R);
  ktime_end(rslot, KT_GEMM_REDUCE, (double)need, st);
  return check_launch("gemm_group_reduce_kernel");
}

// SMI_BWD_DW=0: the BPTT and the heads' weight gradients as separate launches
// (A/B knob); SMI_BWD_DW_EXCL=0: let the two kinds of workgroups share CUs
static bool use_bwd_dw() {
  static const bool on = [] { const char* e = getenv("SMI_BWD_DW"); return !(e && e[0] == '0'); }();
  return on;
}

int launch_lstm_bwd_dw(const float* dh, const float* gates, const float* cbuf, const float* w_hh,
                       int S, int B, int H, float* dgates, hipStream_t st, const int* skip) {
  const int br = lstm_bwd_q_form(B, H, w_hh);
  if (!use_bwd_dw() || !g_grp_on || g_pre_on || g_grp.n == 0 || br == 0 || S <= 0 || B <= 0)
    return SMI_E_NOFIT;
  int cus = 0, dev = 0;
  (void)hipGetDevice(&dev);
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) cus = 256;
  if (cus - B < 32) return SMI_E_NOFIT;             // too few CUs left beside the recurrence
  DwGroup Ga = g_grp;
  int64_t need = 0;
  // balanced for the CUs the recurrence leaves idle (a fixed one-round target
  // of cus - B workgroups with equal slabs: 50.6 vs 30.9 us per launch at 128
  // segments — slab rounding pushed the count past one round)
  RC_CHECK(dw_prepare(Ga, 8, cus - B, 0, need));
  // one workgroup per CU (the LDS request): the recurrence's workgroups keep
  // their CUs to themselves, the weight gradients take the others
  static const bool excl = [] { const char* e = getenv("SMI_BWD_DW_EXCL"); return !(e && e[0] == '0'); }();
  size_t lds = excl ? std::max(kDwdLds, (size_t)84 * 1024) : kDwdLds;
  // the BPTT workgroups stage their step inputs in the same dynamic LDS
  const size_t stg = (size_t)lstm_bwd_stage_floats(S, H) * 4;
  const bool stage = use_bwd_stage() && stg <= kBwdStageMax;
  if (stage) lds = std::max(lds, stg);
  LstmBwdArgs la{dh, gates, cbuf, w_hh, S, B, H, dgates, skip};
  const dim3 grid((unsigned)(B + Ga.wg0[Ga.n]));
  const int kslot = ktime_begin(st);
#define SMI_BD(BR_)                                                                          \
  do {                                                                                       \
    if (stage) {                                                                             \
      allow_lds(lstm_bwd_dw_kernel<BR_, true>, lds);                                         \
      hipLaunchKernelGGL((lstm_bwd_dw_kernel<BR_, true>), grid, dim3(kVT), lds, st, la, Ga); \
    } else {                                                                                 \
      allow_lds(lstm_bwd_dw_kernel<BR_, false>, lds);                                        \
      hipLaunchKernelGGL((lstm_bwd_dw_kernel<BR_, false>), grid, dim3(kVT), lds, st, la, Ga);\
    }                                                                                        \
  } while (0)
  if (br == 16) SMI_BD(16);
  else if (br == 25) SMI_BD(25);
  else SMI_BD(32);
#undef SMI_BD
  ktime_end(kslot, KT_LSTM_BWD, 8.0 * B * H * (double)H * (S - 1), st);
  RC_CHECK(check_launch("lstm_bwd_dw_kernel"));
  g_pre = Ga;
  g_pre_on = true;
  g_pre_need = need;
  workspace_reserve(need);     // no launch before the flush may reuse these partials
  g_grp.n = 0;                                      // the group queues the rest
  g_grp_flops = 0.0;                                // (its launch times the rest only)
  return SMI_OK;
}

static int use_panel() {
  static int u = -1;
  if (u < 0) {
    const char* e = getenv("SMI_PANEL");
    u = (e && e[0] == '0') ? 0 : 1;
  }
  return u;
}

template <int EPI>
static void panel_dispatch(const GemmArgs& g, dim3 grid, int ntw, hipStream_t st) {
  switch (ntw) {
    case 1: hipLaunchKernelGGL((gemm_panel_kernel<EPI, 1>), grid, dim3(kWG), 0, st, g); break;
    case 2: hipLaunchKernelGGL((gemm_panel_kernel<EPI, 2>), grid, dim3(kWG), 0, st, g); break;
    case 4: hipLaunchKernelGGL((gemm_panel_kernel<EPI, 4>), grid, dim3(kWG), 0, st, g); break;
    case 5: hipLaunchKernelGGL((gemm_panel_kernel<EPI, 5>), grid, dim3(kWG), 0, st, g); break;
    case 7: hipLaunchKernelGGL((gemm_panel_kernel<EPI, 7>), grid, dim3(kWG), 0, st, g); break;
    default: hipLaunchKernelGGL((gemm_panel_kernel<EPI, 10>), grid, dim3(kWG), 0, st, g); break;
  }
}

// tall forward / input-gradient GEMMs with 16-byte operands: gemm_panel_kernel
static bool panel_ok(int epi, const GemmArgs& g) {
  auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  // below panel_min_rows the row panels cannot fill the GPU and their serial K
  // loop is the latency: the tiled kernel with split-K takes those (measured at
  // 128 segments per GPU, 2688 / 3328 rows: forwards + input gradients 2.43 ->
  // 1.69 ms per learn, +0.72 ms of split-K reduces, learn 6.10 -> 5.81 ms;
  // SMI_PANEL_MIN_ROWS overrides)
  static const int panel_min_rows = [] {
    const char* e = getenv("SMI_PANEL_MIN_ROWS");
    return e ? atoi(e) : 4096;
  }();
  if (!use_panel() || g.M < panel_min_rows || g.N > 640 || g.K > 1024 || g.K < 1) return false;
  if (g.a_cs != 1 || g.a_rs % 4 || g.K % 4 || !al16(g.A) || !al16(g.B)) return false;
  if (epi == EPI_FWD) return g.b_rs == 1 && g.b_cs % 4 == 0;
  // input gradients: the transposing LDS stage costs more than it saves below
  // ~96 output columns (in the C3 learner 300->100 runs 16 % faster here than
  // on gemm_kernel; SMI_PANEL_DX_MIN overrides)
  static const int dx_min = [] {
    const char* e = getenv("SMI_PANEL_DX_MIN");
    return e ? atoi(e) : 96;
  }();
  if (epi == EPI_DX)
    return g.b_cs == 1 && g.b_rs % 4 == 0 && g.N % 4 == 0 && g.N >= dx_min;
  return false;
}

static int panel_launch(int epi, const GemmArgs& g, hipStream_t st) {
  // column-group width: fewest padded 16-column tiles, then fewer groups
  static const int cand[6] = {1, 2, 4, 5, 7, 10};
  const int t16 = (g.N + 15) / 16;
  int best = 10;
  double bcost = 1e30;
  for (int c : cand) {
    const int groups = (t16 + c - 1) / c;
    const double cost = groups * c + 0.3 * groups;
    if (cost < bcost) { bcost = cost; best = c; }
  }
  const dim3 grid((g.M + 63) / 64, (g.N + 16 * best - 1) / (16 * best), 1);
  const int kslot = ktime_begin(st);
  if (epi == EPI_FWD) panel_dispatch<EPI_FWD>(g, grid, best, st);
  else panel_dispatch<EPI_DX>(g, grid, best, st);
  ktime_end(kslot, epi == EPI_FWD ? KT_GEMM_FWD : KT_GEMM_DX, 2.0 * g.M * (double)g.N * g.K, st);
  return check_launch("gemm_panel_kernel");
}

// Input gradient through a layer with at most 8 outputs (the value head's
// 200 -> 1, the action head's 200 -> 8): dX = (dY W) * [mask > 0] is a
// rank-<=8 update, pure streaming (read dY row + mask, write dX), so it skips
// the MFMA tiles (which pad K to 16/32).  Per element: the k-ordered fmaf
// chain from 0 (for K = 1 bit-identical to the tiled path).  A thread owns 4
// consecutive columns of 4 rows (the W slice in registers, 16-byte mask reads
// and stores, coalesced along the row).  SMI_DX_SMALLK=0 disables it.
template <int KK, bool V4, bool A4 = false>
__global__ void __launch_bounds__(kWG)
dx_smallk_kernel(GemmArgs g) {
  if (g.skip && g.skip[0] != 0) return;
  constexpr int RW = 4;                            // rows per thread
  const int nq = (g.N + 3) >> 2;
  const int64_t idx = (int64_t)blockIdx.x * kWG + threadIdx.x;
  if (idx >= (int64_t)((g.M + RW - 1) / RW) * nq) return;
  const int mg = (int)(idx / nq), n0 = (int)(idx - (int64_t)mg * nq) * 4;
  // W rows k (4 columns each), shared by the thread's RW rows
  float w[KK][4];
#pragma unroll
  for (int k = 0; k < KK; ++k) {
    const float* wr = g.B + (int64_t)min(k, g.K - 1) * g.b_rs;
    if constexpr (V4) {
      const float4 x = *reinterpret_cast<const float4*>(wr + n0);
      w[k][0] = x.x; w[k][1] = x.y; w[k][2] = x.z; w[k][3] = x.w;
    } else {
#pragma unroll
      for (int t = 0; t < 4; ++t) w[k][t] = wr[min(n0 + t, g.N - 1)];
    }
  }
#pragma unroll
  for (int r = 0; r < RW; ++r) {
    const int m = mg * RW + r;
    if (m >= g.M) break;
    const float* arow = g.A + (int64_t)m * g.a_rs;
    float av[KK];
    if (KK % 4 == 0 && A4) {                       // K == KK: 16-byte row loads
#pragma unroll
      for (int q = 0; q < KK / 4; ++q) {
        const float4 x = reinterpret_cast<const float4*>(arow)[q];
        av[4 * q] = x.x; av[4 * q + 1] = x.y; av[4 * q + 2] = x.z; av[4 * q + 3] = x.w;
      }
    } else {
#pragma unroll
      for (int k = 0; k < KK; ++k) av[k] = k < g.K ? arow[k] : 0.f;
    }
    float v[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < KK; ++k) {
      if (k >= g.K) break;
#pragma unroll
      for (int t = 0; t < 4; ++t) v[t] = fmaf(av[k], w[k][t], v[t]);
    }
    const float* mrow = g.mask ? g.mask + (int64_t)m * g.ldm + n0 : nullptr;
    float* crow = g.C + (int64_t)m * g.ldc + n0;
    if constexpr (V4) {
      if (mrow) {
        const float4 mk = *reinterpret_cast<const float4*>(mrow);
        v[0] = mk.x > 0.f ? v[0] : 0.f; v[1] = mk.y > 0.f ? v[1] : 0.f;
        v[2] = mk.z > 0.f ? v[2] : 0.f; v[3] = mk.w > 0.f ? v[3] : 0.f;
      }
      *reinterpret_cast<float4*>(crow) = float4{v[0], v[1], v[2], v[3]};
    } else {
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        if (n0 + t >= g.N) break;
        crow[t] = (mrow && !(mrow[t] > 0.f)) ? 0.f : v[t];
      }
    }
  }
}

static int use_dx_smallk() {
  static int u = -1;
  if (u < 0) {
    const char* e = getenv("SMI_DX_SMALLK");
    u = (e && e[0] == '0') ? 0 : 1;
  }
  return u;
}

static int dx_smallk_launch(const GemmArgs& g, hipStream_t st) {
  auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  const bool v4 = g.N % 4 == 0 && g.ldc % 4 == 0 && al16(g.C) && g.b_rs % 4 == 0 && al16(g.B) &&
                  (!g.mask || (g.ldm % 4 == 0 && al16(g.mask)));
  const int64_t n = (int64_t)((g.M + 3) / 4) * ((g.N + 3) / 4);
  const dim3 grid((unsigned)((n + kWG - 1) / kWG));
  const int kslot = ktime_begin(st);
#define SMI_DXS(KK)                                                                        \
  do {                                                                                     \
    if (v4) hipLaunchKernelGGL((dx_smallk_kernel<KK, true>), grid, dim3(kWG), 0, st, g);   \
    else hipLaunchKernelGGL((dx_smallk_kernel<KK, false>), grid, dim3(kWG), 0, st, g);     \
  } while (0)
  const bool a4 = (g.K == 4 || g.K == 8) && g.a_rs % 4 == 0 && al16(g.A);
  if (g.K == 1) SMI_DXS(1);
  else if (g.K <= 2) SMI_DXS(2);
  else if (g.K == 8 && a4 && v4) hipLaunchKernelGGL((dx_smallk_kernel<8, true, true>), grid, dim3(kWG), 0, st, g);
  else if (g.K <= 4) SMI_DXS(4);
  else SMI_DXS(8);
#undef SMI_DXS
  ktime_end(kslot, KT_GEMM_DX, 2.0 * g.M * (double)g.N * g.K, st);
  return check_launch("dx_smallk_kernel");
}

// Forwards and input gradients of short batches (M <= 4096 rows: DDPG's 512-row
// layers) in ONE launch without split-K: a workgroup owns one 16 x 16 output
// tile and its four waves split K (wave w takes the 16-k chunks c = w, w + 4,
// ...), every chunk's operands loaded up front (one memory round trip), a
// fixed-order LDS sum of the four waves' accumulators, then the epilogue (bias
// + activation, or the input gradient's ReLU mask).  Lane (i, q) = (lane & 15,
// lane >> 4) takes k = 16c + 4q + s at MFMA s of a chunk on both operands (the
// k order permuted identically: every chunk adds its exact 16-term sum), so a
// k-contiguous operand is one 16-byte load per chunk.  The split-K form this
// replaces needed a second launch (the reducer) and ran a 64 x 64 tile's
// serial K loop per slab.
template <int EPI>
__global__ void __launch_bounds__(kWG)
gemm_t16_kernel(GemmArgs g) {
  if (g.skip && g.skip[0] != 0) return;
  __shared__ f32x4 red[4][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int i = lane & 15, q = lane >> 4;
  const int m0 = blockIdx.x * 16, n0 = blockIdx.y * 16;
  const int ra = min(m0 + i, g.M - 1), cb = min(n0 + i, g.N - 1);
  const float* Ar = g.A + (int64_t)ra * g.a_rs;
  const float* Bc = g.B + (int64_t)cb * g.b_cs;
  const int nch = (g.K + 15) >> 4;
  // 16-byte k runs only where k is the contiguous direction (avec / bvec are
  // also set for the other orientation)
  const bool a4 = g.avec && g.a_cs == 1, b4 = g.bvec && g.b_rs == 1;
  float av[T16_MAXC][4], bv[T16_MAXC][4];
#pragma unroll
  for (int j = 0; j < T16_MAXC; ++j) {
    const int c = wave + 4 * j;
    const int k0 = 16 * c + 4 * q;
    if (c >= nch) break;
    if (a4 && k0 + 3 < g.K) {
      const float4 x = *reinterpret_cast<const float4*>(Ar + k0);
      av[j][0] = x.x; av[j][1] = x.y; av[j][2] = x.z; av[j][3] = x.w;
    } else {
#pragma unroll
      for (int t = 0; t < 4; ++t) av[j][t] = k0 + t < g.K ? Ar[(int64_t)(k0 + t) * g.a_cs] : 0.f;
    }
    if (b4 && k0 + 3 < g.K) {
      const float4 x = *reinterpret_cast<const float4*>(Bc + k0);
      bv[j][0] = x.x; bv[j][1] = x.y; bv[j][2] = x.z; bv[j][3] = x.w;
    } else {
#pragma unroll
      for (int t = 0; t < 4; ++t) bv[j][t] = k0 + t < g.K ? Bc[(int64_t)(k0 + t) * g.b_rs] : 0.f;
    }
  }
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j < T16_MAXC; ++j) {
    if (wave + 4 * j >= nch) break;
#pragma unroll
    for (int t = 0; t < 4; ++t) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[j][t], bv[j][t], acc, 0, 0, 0);
  }
  red[wave][lane] = acc;
  __syncthreads();
  if (EPI == EPI_FWD && wave == 1 && blockIdx.y == 0 && g.xsrc) {
    for (int e = lane; e < 16 * g.xcols; e += 64) {
      const int r = e / g.xcols, j = e - r * g.xcols;
      if (m0 + r < g.M) g.C[(int64_t)(m0 + r) * g.ldc + g.N + j] = g.xsrc[(int64_t)(m0 + r) * g.xlds + j];
    }
  }
  if (wave != 0) return;
  const f32x4 sum = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
  // D(row 4q + r, col i)
  const int n = n0 + i;
  if (n >= g.N) return;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int m = m0 + 4 * q + r;
    if (m >= g.M) continue;
    float v = sum[r];
    if constexpr (EPI == EPI_FWD) {
      if (g.bias) v += g.bias[n];
      if (g.act == ACT_RELU) v = v > 0.f ? v : 0.f;
      else if (g.act == ACT_TANH) v = tanhf(v);
    } else {
      if (g.mask && !(g.mask[(int64_t)m * g.ldm + n] > 0.f)) v = 0.f;
    }
    g.C[(int64_t)m * g.ldc + n] = v;
  }
}


static int gemm_launch(int epi, GemmArgs g, hipStream_t st) {
  if (g.M <= 0 || g.N <= 0) return SMI_OK;
  g.part = nullptr;
  if (epi == EPI_DX && use_dx_smallk() && g.K >= 1 && g.K <= 8 && g.a_cs == 1 && g.b_cs == 1)
    return dx_smallk_launch(g, st);
  if (epi != EPI_DW && !g.xsrc && panel_ok(epi, g)) return panel_launch(epi, g, st);
  if (epi == EPI_DW) {
    const bool grp_ok = use_dwd() && g.a_rs == 1 && g.b_cs == 1 && g.K >= 1 &&
                        (g.ones_col >= 0 ? g.ones_col : g.N) >= 1 && g.M <= 512 && g.N <= 512;
    if (grp_ok && dw_group_add(g)) return SMI_OK;
    if (g_grp_on) g_grp_missed = true;     // runs outside the open group
    if (grp_ok) return dwd_launch(g, st);
  }
  const bool ak = g.a_cs == 1;         // A contiguous along k
  const bool bk = g.b_rs == 1;         // B contiguous along k (rows n)
  auto al16 = [](const float* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  // VEC needs the contiguous extent and the other stride in multiples of 4
  // (every K-slab boundary is then a multiple of 4 too: kchunk % 32 == 0)
  g.avec = al16(g.A) && (ak ? (g.K % 4 == 0 && g.a_rs % 4 == 0) : (g.a_rs == 1 && g.M % 4 == 0 && g.a_cs % 4 == 0));
  const int bdata = g.ones_col >= 0 ? g.ones_col : g.N;
  g.bvec = al16(g.B) && (bk ? (g.K % 4 == 0 && g.b_cs % 4 == 0) : (g.b_cs == 1 && bdata % 4 == 0 && g.b_rs % 4 == 0));
  // 128x128 weight-gradient tiles when both operands are row-contiguous
  // float4-able slabs and the output is large enough to need them
  const int breal = g.ones_col >= 0 ? g.ones_col : g.N;
  const bool dw128 = epi == EPI_DW && !ak && !bk && g.a_rs == 1 && g.b_cs == 1 &&
                     al16(g.A) && al16(g.B) && g.M % 4 == 0 && breal % 4 == 0 &&
                     g.a_cs % 4 == 0 && g.b_rs % 4 == 0 && g.M >= 96 && g.N >= 96 &&
                     g.K >= 1024;
  const int TM = dw128 ? D2_T : GBM, TN = dw128 ? D2_T : GBN;
  const int gm = (g.M + TM - 1) / TM, gn = (g.N + TN - 1) / TN;
  int S = 1;
  g.part = nullptr;
  g.kchunk = g.K > 0 ? g.K : 1;
  // split-K: weight gradients (K = rows), and forwards / input gradients whose
  // output has too few tiles to fill the GPU over K >= 128 (the pixel stem's
  // 2592 -> 256 FC; DDPG's 512-row layers: 40 tiles, a serial K loop per tile
  // otherwise; C4 +20 %).  The reducer applies bias/activation or the ReLU mask.
  static const int fwd_split_min = [] {
    const char* e = getenv("SMI_FWD_SPLITK_MIN");
    return e ? atoi(e) : 4 * GBK;
  }();
  const bool split_fwd = (epi == EPI_FWD || epi == EPI_DX) && gm * gn < 256 &&
                         g.K >= fwd_split_min;
  // the short-batch kernel for every forward / input gradient whose 64 x 64
  // tiling leaves the GPU mostly idle (< 256 tiles), split-K or not
  if ((epi == EPI_FWD || epi == EPI_DX) && gm * gn < 256 && use_t16() && g.M <= 4096 &&
      g.K <= 4 * 16 * T16_MAXC) {
    const dim3 grid16((g.M + 15) / 16, (g.N + 15) / 16);
    const int kslot = ktime_begin(st);
    if (epi == EPI_FWD) hipLaunchKernelGGL(gemm_t16_kernel<EPI_FWD>, grid16, dim3(kWG), 0, st, g);
    else hipLaunchKernelGGL(gemm_t16_kernel<EPI_DX>, grid16, dim3(kWG), 0, st, g);
    ktime_end(kslot, epi == EPI_FWD ? KT_GEMM_FWD : KT_GEMM_DX, 2.0 * g.M * (double)g.N * g.K, st);
    return check_launch("gemm_t16_kernel");
  }
  if ((epi == EPI_DW && g.K > 4 * GBK) || split_fwd) {
    const int tiles = gm * gn;
    S = (smi_splitk_target() + tiles - 1) / tiles;    // ~2-4 workgroups per CU
    const int smax = (g.K + 4 * GBK - 1) / (4 * GBK);   // >= 4 K-steps per slab
    if (S > smax) S = smax;
    const int64_t cap = smi_workspace_floats() / ((int64_t)g.M * g.N);
    if (S > cap) S = (int)cap;
    if (S < 1) S = 1;
    // one MFMA chain per slab: <= 512 rows (longer fixed slabs measured slower:
    // fewer workgroups in flight outweigh the smaller partial traffic)
    if (dw128 && (g.K + S - 1) / S > 512) S = (g.K + 511) / 512;
    if (S > cap) S = (int)cap;
    if (S < 1) S = 1;
    if (S > 1) {
      g.kchunk = ((g.K + S - 1) / S + 31) / 32 * 32;
      S = (g.K + g.kchunk - 1) / g.kchunk;
      g.part = workspace_f32((int64_t)S * g.M * g.N);
      if (!g.part) return set_error(SMI_E_ARG, "gemm: workspace unavailable for split-K");
    }
  }
  const dim3 grid(gm, gn, S);
  const int kslot = ktime_begin(st);
  if (dw128) hipLaunchKernelGGL(gemm_dw128_kernel, grid, dim3(kWG), 0, st, g);
  else if (epi == EPI_FWD) gemm_dispatch<EPI_FWD>(g, grid, ak, bk, st);
  else if (epi == EPI_DX) gemm_dispatch<EPI_DX>(g, grid, ak, bk, st);
  else gemm_dispatch<EPI_DW>(g, grid, ak, bk, st);
  const int nreal = g.ones_col >= 0 ? g.N - 1 : g.N;
  ktime_end(kslot, epi == EPI_FWD ? KT_GEMM_FWD : epi == EPI_DX ? KT_GEMM_DX : KT_GEMM_DW,
            2.0 * g.M * (double)nreal * g.K + (g.ones_col >= 0 ? (double)g.M * g.K : 0.0), st);
  int rc = check_launch("gemm_kernel");
  if (rc || S == 1) return rc;
  return splitk_reduce(g, S, epi, st);
}

static int splitk_reduce(const GemmArgs& g, int S, int epi, hipStream_t st) {
  const int rslot = ktime_begin(st);
  const int64_t MN = (int64_t)g.M * g.N;
  const int rg = (int)((MN + 63) / 64);
  const bool fwd = epi == EPI_FWD;
  hipLaunchKernelGGL(gemm_splitk_reduce_kernel, dim3(rg), dim3(kWG), 0, st, g.part, S, g,
                     fwd ? g.bias : nullptr, fwd ? g.act : ACT_NONE,
                     epi == EPI_DX ? g.mask : nullptr);
  ktime_end(rslot, KT_GEMM_REDUCE, (double)S * MN, st);
  return check_launch("gemm_splitk_reduce_kernel");
}

// out[i] = sum_{z < S} part[z][i] in a fixed order (no accumulate)
int launch_slab_reduce(const float* part, int S, int64_t n, float* out, hipStream_t st,
                       const int* skip) {
  if (n < 1 || S < 1) return SMI_OK;
  const int rg = (int)((n + 63) / 64);
  GemmArgs g{};
  g.M = 1; g.N = (int)n; g.C = out; g.ldc = n; g.ones_col = -1; g.skip = skip;
  hipLaunchKernelGGL(gemm_splitk_reduce_kernel, dim3(rg), dim3(kWG), 0, st, part, S, g, nullptr,
                     ACT_NONE, nullptr);
  return check_launch("gemm_splitk_reduce_kernel");
}

int launch_linear_fwd(const float* X, int64_t ldx, int M, int K, const float* W, int64_t ldw,
                      const float* b, int N, int act, float* Y, int64_t ldy, hipStream_t st,
                      const int* skip) {
  if (K >= 1 && K <= 64 && N >= 32 && N <= 512 && M >= 2048)
    return launch_smallk_fwd(X, ldx, M, K, W, ldw, b, N, act, Y, ldy, st, skip);
  GemmArgs g{};
  g.M = M; g.N = N; g.K = K;
  g.A = X; g.a_rs = ldx; g.a_cs = 1;
  g.B = W; g.b_rs = 1; g.b_cs = ldw;        // B(k,n) = W[n][k]
  g.C = Y; g.ldc = ldy; g.bias = b; g.act = act; g.ones_col = -1; g.skip = skip;
  return gemm_launch(EPI_FWD, g, st);
}

// launch_linear_fwd plus Y[:, N : N + xcols] = S[:, :xcols] (one launch on the
// short-batch kernel, else the forward and a column copy)
int launch_copy_cols(const float* src, int64_t lds, int64_t rows, int cols, float* dst,
                     int64_t ldd, hipStream_t st);
int launch_linear_fwd_cat(const float* X, int64_t ldx, int M, int K, const float* W, int64_t ldw,
                          const float* b, int N, int act, float* Y, int64_t ldy, const float* S,
                          int64_t lds, int xcols, hipStream_t st) {
  const int gm = (M + GBM - 1) / GBM, gn = (N + GBN - 1) / GBN;
  const bool t16 = !(K >= 1 && K <= 64 && N >= 32 && N <= 512 && M >= 2048) && use_t16() &&
                   gm * gn < 256 && M <= 4096 && K <= 4 * 16 * T16_MAXC && M > 0;
  if (!t16) {
    RC_CHECK(launch_linear_fwd(X, ldx, M, K, W, ldw, b, N, act, Y, ldy, st));
    return launch_copy_cols(S, lds, M, xcols, Y + N, ldy, st);
  }
  GemmArgs g{};
  g.M = M; g.N = N; g.K = K;
  g.A = X; g.a_rs = ldx; g.a_cs = 1;
  g.B = W; g.b_rs = 1; g.b_cs = ldw;
  g.C = Y; g.ldc = ldy; g.bias = b; g.act = act; g.ones_col = -1;
  g.xsrc = S; g.xlds = lds; g.xcols = xcols;
  return gemm_launch(EPI_FWD, g, st);
}

int launch_linear_bwd_dx(const float* dY, int64_t ldg, int M, int N, const float* W, int64_t ldw,
                         int K, const float* mask, int64_t ldm, float* dX, int64_t lddx,
                         hipStream_t st, const int* skip) {
  GemmArgs g{};
  g.M = M; g.N = K; g.K = N;
  g.A = dY; g.a_rs = ldg; g.a_cs = 1;
  g.B = W; g.b_rs = ldw; g.b_cs = 1;        // B(k=n', n=k') = W[n'][k']
  g.C = dX; g.ldc = lddx; g.mask = mask; g.ldm = ldm; g.ones_col = -1; g.skip = skip;
  return gemm_launch(EPI_DX, g, st);
}

// weight gradients of two layers fed by the same dY over [X1 | X2] (the LSTM:
// W_ih over x_t, W_hh over h_{t-1}, one bias gradient shared by b_ih / b_hh)
// in ONE launch: dY read once, one split-K reduce.  X1 has K1 real columns and
// row stride ldx1 (a multiple of 4 >= K1: the padding columns are computed and
// dropped so both sources load as 16-byte vectors).
int launch_linear_bwd_dw2(const float* dY, int64_t ldg, int M, int N, const float* X1,
                          int64_t ldx1, int K1, const float* X2, int64_t ldx2, int K2,
                          float* dW1, int64_t ld1, float* dW2, int64_t ld2, float* db1,
                          float* db2, hipStream_t st, const int* skip) {
  const int K1p = (int)ldx1;
  if (K1p < K1 || K1p % 4) return set_error(SMI_E_ARG, "bwd_dw2: ldx1 must be a multiple of 4 >= K1");
  GemmArgs g{};
  g.M = N; g.N = K1p + K2 + 1; g.K = M;
  g.A = dY; g.a_rs = 1; g.a_cs = ldg;
  g.B = X1; g.b_rs = ldx1; g.b_cs = 1;
  g.B2 = X2; g.b2_rs = ldx2; g.split_col = K1p; g.c1_real = K1;
  g.C = dW1; g.ldc = ld1; g.C2 = dW2; g.ldc2 = ld2;
  g.ones_col = K1p + K2; g.bias_out = db1; g.bias_out2 = db2; g.skip = skip;
  if (!(g.a_rs == 1 && g.b_cs == 1 && use_dwd() && g.M <= 512 && g.N <= 512))
    return set_error(SMI_E_ARG, "bwd_dw2: shape not supported");
  if (dw_group_add(g)) return SMI_OK;
  if (g_grp_on) g_grp_missed = true;
  return dwd_launch(g, st);
}

int launch_linear_bwd_dw(const float* dY, int64_t ldg, int M, int N, const float* X, int64_t ldx,
                         int K, float* dW, int64_t lddw, float* db, int accumulate,
                         hipStream_t st, const int* skip) {
  GemmArgs g{};
  g.M = N; g.N = db ? K + 1 : K; g.K = M;
  g.A = dY; g.a_rs = 1; g.a_cs = ldg;       // A(m=n, k=r) = dY[r][n]
  g.B = X; g.b_rs = ldx; g.b_cs = 1;        // B(k=r, n=k') = X[r][k'] (k' == K: 1)
  g.C = dW; g.ldc = lddw; g.accumulate = accumulate; g.skip = skip;
  g.ones_col = db ? K : -1;
  g.bias_out = db;
  return gemm_launch(EPI_DW, g, st);
}

}  // namespace smi
