// head_kernels.hip — the PPO actor / critic MLP heads over the learner's tall
// activation matrices (builders.py:86-175: Linear-ReLU-Linear-ReLU-Linear
// [-Tanh], PPO_ActorNetwork / PPO_CriticNetwork; ppo_net.py:143-152,277-315
// feed them the LSTM outputs), the forward and the input-gradient chain each
// as ONE launch instead of three GEMM launches (+ split-K reduces at small
// batches).
//
// A workgroup owns 16 rows (one MFMA row tile) and runs every layer of the
// chain over them; the activations between layers stay in LDS, the weights
// stream from L2 straight into MFMA registers.  Layer Y = X W^T with W [N][K]
// row-major (k contiguous):
//   * output features in 16-column tiles, tile nt on wave nt % 4;
//   * k in chunks of 16: lane (li, lk) reads X[li][16c + 4lk .. +3] from LDS
//     and W[16 nt + li][16c + 4lk .. +3] from global memory (16-byte reads),
//     and MFMA j of the chunk (v_mfma_f32_16x16x4_f32) takes element j of
//     both: the k order inside a chunk is permuted identically on the two
//     operands, so every chunk adds its exact 16-term dot product (an fmaf
//     chain, like every f32 MFMA);
//   * the weight reads of the next two chunks are in flight behind the MFMAs
//     of the current one (register ring, sched_barrier pins the refills);
//   * the epilogue (bias + ReLU, or the ReLU mask of the backward) writes the
//     tile to LDS for the next layer and the workgroup copies the rows out to
//     HBM as 16-byte stores (HA1 / HA2 for the backward, dH2 / dH1 for the
//     weight gradients).
// The narrow last layer (<= 16 outputs: the 8 action means, the value) splits
// its k chunks over the four waves and sums the four partials in a fixed order.
//
// The backward chain dH2 = (dZ W3) * [HA2 > 0], dH1 = (dH2 W2) * [HA1 > 0],
// dX = dH1 W1[:, cols] reads W2 and W1 TRANSPOSED (k contiguous again): the
// forward of the same phase writes W1^T and W2^T as a side job (the weights do
// not change between a phase's forward and backward), so the backward's
// weight reads are 16-byte reads too.  dZ W3 has K = out <= 16 (8 actions or
// the value): a VALU pass in the order of the streaming small-K kernel.
//
// Rows are the learner's [step][segment] rows; the weight gradients of the
// three layers stay in the phase's grouped dW launch (linear_kernels.hip).
#include "smi_device.hpp"
#include "smi_internal.hpp"
#include "pol_rows.hpp"

namespace smi {

constexpr int HC_R = 16;                 // rows per workgroup
constexpr int HC_MAXK = 512;             // widest layer input / output handled here
constexpr int HC_SR = 32 * 33 + 32;     // last-layer partials (1024) / a transpose tile (1056)

struct HeadFwdArgs {
  const float* X; int64_t ldx; int K0;   // input rows [rows][ldx], K0 features
  const float* W1; const float* b1;      // [h1][K0]
  const float* W2; const float* b2;      // [h2][h1]
  const float* W3; const float* b3;      // [out][h2]
  int h1, h2, out, tanh_out;
  float* HA1; float* HA2;                // [rows][h1], [rows][h2] (post-ReLU)
  float* Y; int64_t ldy;                 // [rows][ldy]
  float* W1T; float* W2T;                // optional: [K0][h1], [h1][h2] for the backward
  int64_t rows; const int* skip;
  int ld0, ld1, ld2;                     // LDS leading dims (floats)
  // optional value-loss epilogue (out == 1, ppo.py:311-331): vgrad[r] =
  // vscale * (Y[r] - vret[r]), the MSE gradient the learner's value_rows pass
  // would compute from Y (same fp32 ops), written by the forward itself
  const float* vret; float* vgrad; float vscale;
  // policy statistics epilogue (head_fwd_kernel<..., PS>, adapt mode, out ==
  // 8): the rows' sums of policy_rows_stats_kernel's pass from the means the
  // forward just formed, one PS_N partial per workgroup at ps.part
  PolRowArgs ps;
  // with vgrad: the value statistics of the last value epoch (ppo.py:324-331,
  // value_rows_kernel's sums {sum (V-R)^2, sum (R-V), sum (R-V)^2, sum R,
  // sum R^2}), five fp64 per workgroup at vpart[blockIdx.x * 5 ..] (nullable)
  double* vpart;
};

struct HeadBwdArgs {
  const float* dZ; int out;              // [rows][out]: gradient at the last pre-activation
  const float* W3;                       // [out][h2]
  const float* W2T;                      // [h1][h2] (forward's transpose)
  const float* W1T;                      // [in][h1] (forward's transpose)
  int h1, h2, dx0, dxn;                  // dX columns [dx0, dx0 + dxn) of the head input
  const float* HA1; const float* HA2;    // forward activations (ReLU masks)
  float* dH2; float* dH1;                // [rows][h2], [rows][h1]
  float* dX; int64_t lddx;               // [rows][lddx]
  const float* mask; int64_t ldm;        // optional: dX zero where mask <= 0
  int64_t rows; const int* skip;
  int ld2, ld1;                          // LDS leading dims
  // policy-gradient prologue (head_bwd_kernel<..., PG>): dZ of the workgroup's
  // rows computed here from the policy rows (policy_rows_grad_kernel's pass)
  // instead of read; written to pg.dz for the layer-3 weight gradient, the
  // rows' d/dstd sums to pg.lvpart[blockIdx.x]
  PolRowArgs pg;
};

// Developer phase timer (build variant 'prof', -DSMI_PROF): thread 0 of every
// workgroup adds its wall-clock ticks (100 MHz) per phase into g_head_ticks
// (vector atomics), [8] counts the workgroups; forward and backward each own
// 10 slots (smi_head_phase_ticks, tools/head_ticks.py)
#ifdef SMI_PROF
__device__ unsigned long long g_head_ticks[2][10];
#define HEAD_T0() unsigned long long h_t0_ = wall_clock64(), h_prev_ = h_t0_
#define HEAD_TICK(k, id)                                                   \
  do {                                                                      \
    if (threadIdx.x == 0) {                                                 \
      const unsigned long long n_ = wall_clock64();                         \
      atomicAdd(&g_head_ticks[k][id], n_ - h_prev_);                        \
      h_prev_ = n_;                                                         \
    }                                                                       \
  } while (0)
#define HEAD_END(k)                                                        \
  do {                                                                      \
    if (threadIdx.x == 0) {                                                 \
      atomicAdd(&g_head_ticks[k][8], 1ull);                                 \
      atomicAdd(&g_head_ticks[k][9], wall_clock64() - h_t0_);               \
    }                                                                       \
  } while (0)
#else
#define HEAD_T0() (void)0
#define HEAD_TICK(k, id) (void)0
#define HEAD_END(k) (void)0
#endif

// LDS leading dim of a K-wide activation tile: K rounded up to the 16-k chunk,
// + 4 (an odd multiple of 4 floats: the 16 rows of a chunk read land on 16
// distinct 16-byte bank groups)
__host__ __device__ inline int hc_ld(int k) { return ((k + 15) & ~15) + 4; }

// A barrier for LDS hand-offs between the waves only: the fences are limited
// to the LDS address space, so global loads in flight (the next layer's weight
// prefetch) stay in flight across it instead of being drained (a plain
// __syncthreads() waits vmcnt(0))
__device__ __forceinline__ void hc_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// The weight stream of one layer: output tiles nt = nt0 + ntst * t (t < NT,
// nt < ceil(N / 16)) over the k chunks c0, c0 + cst, ... (< ceil(K / 16)),
// through a ring of HC_D chunk slots.  init() issues the weight reads of the
// first two chunks, which need nothing from the layer's input: a layer's init
// runs before the previous layer's epilogue and barrier, so those reads are
// in flight meanwhile; hc_run issues the rest of the ring.
#ifndef SMI_HC_DEPTH
#define SMI_HC_DEPTH 2
#endif
// chunks in flight per wave; measured (C3 bench, one MI355X, interleaved
// trials): 2 -> 8.45 ms, 3 -> 8.59, 4 -> 8.67 per learn: the deeper rings cost
// occupancy (124 -> 184 VGPRs) and gain nothing
constexpr int HC_D = SMI_HC_DEPTH;
// 16-byte X loads per thread in flight while staging the forward's input rows
#ifndef SMI_HC_XB
#define SMI_HC_XB 4
#endif
constexpr int HC_XB = SMI_HC_XB;
static_assert(HC_D >= 2, "ring of at least two chunks");
template <int NT>
struct HcStream {
  const float* wp[NT];
  float4 b[HC_D][NT];
  int K, nch, c0, cst, ntv;
  // k past K (the last chunk of a K % 16 != 0 layer) reads the row's last
  // float4 instead (clamped address: no branch, no select after the load) and
  // meets A = 0 there: the LDS tiles are zero-padded up to the chunk.  Loads
  // are issued unconditionally (chunk indices clamped): a load issued on one
  // path only made the waitcnt pass assume the shorter queue everywhere and
  // wait for nearly every load in flight.
  __device__ __forceinline__ void ldb(int c, float4 (&bb)[NT]) {
    const int lk = (threadIdx.x & 63) >> 4;
    const int kk = min(16 * c + 4 * lk, K - 4);     // K % 4 == 0
#pragma unroll
    for (int t = 0; t < NT; ++t) bb[t] = *reinterpret_cast<const float4*>(wp[t] + kk);
  }
  __device__ __forceinline__ void init(const float* __restrict__ W, int64_t ldw, int K_, int N,
                                       int nt0, int ntst, int c0_, int cst_) {
    const int li = threadIdx.x & 15;
    const int CT = (N + 15) >> 4;
    K = K_; nch = (K + 15) >> 4; c0 = c0_; cst = cst_;
    // tiles of this wave that exist (wave-uniform)
    ntv = __builtin_amdgcn_readfirstlane(nt0 < CT ? (CT - 1 - nt0) / ntst + 1 : 0);
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int n = min(16 * (nt0 + ntst * t) + li, N - 1);
      wp[t] = W + (int64_t)n * ldw;
    }
    ldb(min(c0, nch - 1), b[0]);
    ldb(min(c0 + cst, nch - 1), b[1]);
  }
};

// acc[rt][t] = A[16 rt .. 16 rt + 15][K] (LDS, lda) x W^T over the stream's
// tiles and chunks: RT row tiles share every weight chunk (RT = 2 halves the
// weight traffic per flop at large batches)
template <int NT, int RT, bool CM = false>
__device__ __forceinline__ void hc_run(HcStream<NT>& S, const float* sA, int lda,
                                       f32x4 (&acc)[RT][NT]) {
  const int lane = threadIdx.x & 63, li = lane & 15, lk = lane >> 4;
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[rt][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (S.ntv == 0) return;
  const float* ap = sA + li * lda + 4 * lk;
  // every tile slot runs (a slot past the last tile reads clamped rows and its
  // result is dropped): per-tile guards made the compiler move the
  // accumulators out of AGPRs every chunk.  NT is chosen per layer so that at
  // most one slot per wave is idle.
  // tile major (CM false): each tile's four k components back to back, the
  // row tiles interleaved; k-component major (CM): consecutive MFMAs go to
  // different accumulators.  Each accumulator takes x, y, z, w in order either
  // way (bit-identical sums).  Measured at C3 (interleaved trials): the forward
  // 67.5 (tile major) vs 70.1 us, the input-gradient chain 64.0 vs 62.4 us
  auto mm = [&](const float4 (&a)[RT], const float4 (&bb)[NT]) {
    if constexpr (!CM) {
#pragma unroll
      for (int t = 0; t < NT; ++t) {
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) acc[rt][t] = mfma4(a[rt].x, bb[t].x, acc[rt][t]);
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) acc[rt][t] = mfma4(a[rt].y, bb[t].y, acc[rt][t]);
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) acc[rt][t] = mfma4(a[rt].z, bb[t].z, acc[rt][t]);
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) acc[rt][t] = mfma4(a[rt].w, bb[t].w, acc[rt][t]);
      }
    } else {
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) acc[rt][t] = mfma4(a[rt].x, bb[t].x, acc[rt][t]);
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) acc[rt][t] = mfma4(a[rt].y, bb[t].y, acc[rt][t]);
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) acc[rt][t] = mfma4(a[rt].z, bb[t].z, acc[rt][t]);
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) acc[rt][t] = mfma4(a[rt].w, bb[t].w, acc[rt][t]);
    }
  };
  auto lda_ = [&](int c, float4 (&o)[RT]) {
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
      o[rt] = *reinterpret_cast<const float4*>(ap + rt * 16 * lda + 16 * c);
  };
  const int nch = S.nch, cst = S.cst, cl = nch - 1;
  int c = S.c0;
  float4 a[HC_D][RT];
#pragma unroll
  for (int d = 2; d < HC_D; ++d) S.ldb(min(c + d * cst, cl), S.b[d]);
#pragma unroll
  for (int d = 0; d < HC_D; ++d) lda_(min(c + d * cst, cl), a[d]);
  // steady state without conditionals (HC_D chunks per trip, every refill
  // issued): the waitcnt pass then sees the ring's loads in flight and waits
  // for exactly the slot it consumes
  for (; c + (2 * HC_D - 1) * cst < nch; c += HC_D * cst) {
#pragma unroll
    for (int d = 0; d < HC_D; ++d) {
      mm(a[d], S.b[d]);
      lda_(c + (d + HC_D) * cst, a[d]);
      S.ldb(c + (d + HC_D) * cst, S.b[d]);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  // the last < 2 HC_D chunks
#pragma unroll
  for (int d = 0; d < HC_D; ++d) {
    if (c + d * cst < nch) mm(a[d], S.b[d]);
    lda_(min(c + (d + HC_D) * cst, cl), a[d]);
    S.ldb(min(c + (d + HC_D) * cst, cl), S.b[d]);
  }
#pragma unroll
  for (int d = 0; d < HC_D; ++d)
    if (c + (d + HC_D) * cst < nch) mm(a[d], S.b[d]);
}

// the wave's tiles of a full-width layer into LDS rows: D(row 4lk + i, col li)
// of tile nt, row tile rt, is element [16 rt + 4lk + i][16 nt + li]; EPI 0:
// + bias, ReLU; 1: * [mask > 0] (mask row-major [rows][N] in global memory,
// rows r0..); columns N..16*CT-1 are written as zeros (the next layer's last
// chunk reads them)
// Its operands (the bias, or the 4 mask values of each of the lane's rows)
// are fetched by hc_epi_load BEFORE the layer's k loop, so their latency hides
// behind it instead of serializing one tile at a time after it.  EPI 0 uses
// e[0] only (the bias is the same for every row tile).
template <int NT, int EPI, int RT>
__device__ __forceinline__ void hc_epi_load(int nt0, int N, const float* bias, const float* mask,
                                            int64_t r0, int64_t rows, float (&e)[RT][NT][4]) {
  const int lane = threadIdx.x & 63, li = lane & 15, lk = lane >> 4;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int nc = min(16 * (nt0 + 4 * t) + li, N - 1);     // clamped: unconditional loads
    if constexpr (EPI == 0) {
      e[0][t][0] = bias[nc];
    } else {
#pragma unroll
      for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int64_t r = r0 + 16 * rt + 4 * lk + i;
          e[rt][t][i] = mask[(r < rows ? r : rows - 1) * N + nc];
        }
    }
  }
}

template <int NT, int EPI, int RT>
__device__ __forceinline__ void hc_store(const f32x4 (&acc)[RT][NT], const float (&e)[RT][NT][4],
                                         int nt0, int N, float* sO, int ldo) {
  const int lane = threadIdx.x & 63, li = lane & 15, lk = lane >> 4;
  const int CT = (N + 15) >> 4;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int nt = nt0 + 4 * t;
    if (nt >= CT) break;
    const int n = 16 * nt + li;
    const bool nv = n < N;
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = 16 * rt + 4 * lk + i;
        float v;
        if constexpr (EPI == 0) {
          v = acc[rt][t][i] + e[0][t][0];
          v = v > 0.f ? v : 0.f;
        } else {
          v = e[rt][t][i] > 0.f ? acc[rt][t][i] : 0.f;
        }
        sO[r * ldo + n] = nv ? v : 0.f;
      }
  }
}

// rows r0.. of an LDS tile [16 RT][ld] (N columns, N % 4 == 0, N <= HC_MAXK) to
// global [rows][N]: thread (r, q0) copies row r's float4 columns q0, q0 + 16,
// ... of each row tile; every LDS read of a row tile first, into distinct
// registers, then its stores (a loop reusing one register made each store wait
// for the previous one)
template <int RT>
__device__ __forceinline__ void hc_copy_out(const float* sO, int ld, int N, float* __restrict__ G,
                                           int64_t r0, int64_t rows) {
  if (G == nullptr) return;                      // (no backward reads them: not stored)
  constexpr int J = HC_MAXK / 4 / 16;
  const int nq = N >> 2, q0 = threadIdx.x & 15;
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
    const int r = (threadIdx.x >> 4) + 16 * rt;
    float4 v[J];
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const int q = q0 + 16 * j;
      v[j] = q < nq ? *reinterpret_cast<const float4*>(sO + r * ld + 4 * q) : float4{0.f, 0.f, 0.f, 0.f};
    }
    if (r0 + r >= rows) continue;
    float* g = G + (r0 + r) * N;
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const int q = q0 + 16 * j;
      if (q < nq) *reinterpret_cast<float4*>(g + 4 * q) = v[j];
    }
  }
}

// W [M][K] -> WT [K][M] in 32 x 32 tiles (tile index tix over both matrices)
__device__ __forceinline__ void hc_transpose_tile(const float* __restrict__ W, int M, int K,
                                                  float* __restrict__ WT, int tix, float* sT) {
  const int tk = (K + 31) >> 5;
  const int m0 = (tix / tk) * 32, k0 = (tix % tk) * 32;
  __syncthreads();
  // the tile's loads unconditional (clamped), pinned, then the conditional
  // LDS stores: a load under the bounds test was its own branch with a wait,
  // four round trips per tile (round 6)
  static_assert(32 * 32 % kWG == 0, "whole tile passes");
  constexpr int TP = 32 * 32 / kWG;
  float v[TP];
#pragma unroll
  for (int i = 0; i < TP; ++i) {
    const int e = threadIdx.x + i * kWG, r = e >> 5, c = e & 31;
    v[i] = W[(int64_t)min(m0 + r, M - 1) * K + min(k0 + c, K - 1)];
  }
#pragma unroll
  for (int i = 0; i < TP; ++i) asm volatile("" : "+v"(v[i]));
#pragma unroll
  for (int i = 0; i < TP; ++i) {
    const int e = threadIdx.x + i * kWG, r = e >> 5, c = e & 31;
    if (m0 + r < M && k0 + c < K) sT[r * 33 + c] = v[i];
  }
  __syncthreads();
  for (int e = threadIdx.x; e < 32 * 32; e += kWG) {
    const int r = e >> 5, c = e & 31;           // WT row k0 + r, column m0 + c
    if (k0 + r < K && m0 + c < M) WT[(int64_t)(k0 + r) * M + m0 + c] = sT[c * 33 + r];
  }
}

// LDS floats of the forward's last-layer partials / transpose tile
__host__ __device__ constexpr int hc_sr(int RT) { return RT * 1024 > HC_SR ? RT * 1024 : HC_SR; }

template <int NT1, int NT2, int RT, bool PS>
__global__ void __launch_bounds__(kWG)
head_fwd_kernel(HeadFwdArgs a) {
  if (a.skip && a.skip[0] != 0) return;
  constexpr int R = HC_R * RT;                    // rows per workgroup
  extern __shared__ __attribute__((aligned(16))) float hsm[];
  // X and HA2 share one region (X is dead once layer 1's k loop is done: the
  // barrier after its epilogue orders that before layer 2 writes HA2): 37.5 KB
  // at C3 widths and RT = 1, four workgroups per CU
  float* s0 = hsm;                                // [R][ld0]  X
  float* s2 = hsm;                                // [R][ld2]  HA2
  float* s1 = hsm + R * (a.ld0 > a.ld2 ? a.ld0 : a.ld2);   // [R][ld1]  HA1
  float* sR = s1 + R * a.ld1;                     // [4][RT][64][4] partials of the last layer;
                                                  // [32][33] transpose tile
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63, li = lane & 15, lk = lane >> 4;
  const int64_t r0 = (int64_t)blockIdx.x * R;
  HEAD_T0();
  if (r0 < a.rows) {
    // layer 1's weight stream and bias first: in flight while X arrives
    HcStream<NT1> S1;
    S1.init(a.W1, a.K0, a.K0, a.h1, wave, 4, 0, 1);
    float e1[RT][NT1][4];
    hc_epi_load<NT1, 0, RT>(wave, a.h1, a.b1, nullptr, r0, a.rows, e1);
    // X rows into LDS (columns K0 .. ld0 - 4 zero: the last chunk's padding),
    // HC_XB 16-byte loads per thread in flight before their LDS stores (one
    // memory round trip per batch instead of one per float4; addresses
    // clamped, the padding zeroed at the store)
    const int q0 = (a.ld0 - 4) >> 2;
    for (int e0 = threadIdx.x; e0 < R * q0; e0 += HC_XB * kWG) {
      f32x4 v[HC_XB];
#pragma unroll
      for (int k = 0; k < HC_XB; ++k) {
        const int e = min(e0 + k * kWG, R * q0 - 1);
        const int r = e / q0, q = e - r * q0;
        const int64_t rr = r0 + r < a.rows ? r0 + r : a.rows - 1;
        v[k] = *reinterpret_cast<const f32x4*>(a.X + rr * a.ldx + min(4 * q, a.K0 - 4));
      }
#pragma unroll
      for (int k = 0; k < HC_XB; ++k) {
        const int e = e0 + k * kWG;
        if (e >= R * q0) break;
        const int r = e / q0, q = e - r * q0;
        const f32x4 z = {0.f, 0.f, 0.f, 0.f};
        *reinterpret_cast<f32x4*>(s0 + r * a.ld0 + 4 * q) = 4 * q < a.K0 ? v[k] : z;
      }
    }
    __syncthreads();
    HEAD_TICK(0, 0);                              // X staged
    HcStream<NT2> S2;
    float e2[RT][NT2][4];
    {   // layer 1: HA1 = relu(X W1^T + b1)
      f32x4 acc[RT][NT1];
      // every load before this point has landed (the X rows went through
      // registers into LDS), but on the path where this thread staged no X
      // the waitcnt pass still counts the stream's first chunks and the bias
      // loads in flight, and that merged state set the k loop's header waits
      // to vmcnt(4) / vmcnt(1) instead of the ring depth (vmcnt(9..5)): an
      // explicit vmcnt(0) (expcnt / lgkmcnt left at their maxima) clears it
      __builtin_amdgcn_s_waitcnt(0x0F70);
      hc_run<NT1, RT>(S1, s0, a.ld0, acc);
      HEAD_TICK(0, 1);                            // layer 1 k loop
      S2.init(a.W2, a.h1, a.h1, a.h2, wave, 4, 0, 1);     // layer 2's stream, in flight
      hc_epi_load<NT2, 0, RT>(wave, a.h2, a.b2, nullptr, r0, a.rows, e2);
      hc_store<NT1, 0, RT>(acc, e1, wave, a.h1, s1, a.ld1);
    }
    hc_sync();
    HEAD_TICK(0, 2);                              // epilogue 1 + barrier
    hc_copy_out<RT>(s1, a.ld1, a.h1, a.HA1, r0, a.rows);
    HEAD_TICK(0, 3);                              // HA1 copy-out issue
    HcStream<1> S3;
    {   // layer 2: HA2 = relu(HA1 W2^T + b2)
      f32x4 acc[RT][NT2];
      hc_run<NT2, RT>(S2, s1, a.ld1, acc);
      HEAD_TICK(0, 4);                            // layer 2 k loop
      S3.init(a.W3, a.h2, a.h2, a.out, 0, 1, wave, 4);    // layer 3's stream
      hc_store<NT2, 0, RT>(acc, e2, wave, a.h2, s2, a.ld2);
    }
    hc_sync();
    HEAD_TICK(0, 5);                              // epilogue 2 + barrier
    hc_copy_out<RT>(s2, a.ld2, a.h2, a.HA2, r0, a.rows);
    // PS: thread t < R's row inputs of the statistics pass, in flight through
    // layer 3
    constexpr int R_ = HC_R * RT, PA = 8;
    __shared__ float smu[PS ? R_ * PA : 1];
    float prm[PS ? PA : 1], pac[PS ? PA : 1], pbl = 1.f, prbd = 0.f, padv = 0.f, pret = 0.f;
    const int64_t prow = r0 + threadIdx.x;
    const bool pown = PS && (int)threadIdx.x < R_ && prow < a.rows;
    if constexpr (PS) {
      if (pown) {
        const int64_t N = (int64_t)a.ps.E * a.ps.B;
        ld_row<PA>(prm, a.ps.refmu + prow * PA, PA);
        ld_fields<PA>(pac, a.ps.rowin, N, prow, 0, PA);
        padv = a.ps.rowin[rin_idx(row_w(PA), prow, rin_adv(PA))];
        pbl = a.ps.rowin[rin_idx(row_w(PA), prow, rin_bl(PA))];
        prbd = a.ps.rowin[rin_idx(row_w(PA), prow, rin_rbd(PA))];
        pret = a.ps.ret_tm[prow];
      }
    }
    {   // layer 3 (out <= 16): the waves split the k chunks, fixed-order sum
      const float bn = a.b3[li < a.out ? li : a.out - 1];
      // the value targets of the lane's rows (value-gradient epilogue), in
      // flight through layer 3
      float vr[RT][4];
      if (a.vgrad) {
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
          for (int i = 0; i < 4; ++i)
            vr[rt][i] = a.vret[min(r0 + 16 * rt + 4 * lk + i, a.rows - 1)];
      }
      f32x4 acc[RT][1];
      hc_run<1, RT>(S3, s2, a.ld2, acc);
#pragma unroll
      for (int rt = 0; rt < RT; ++rt)
        *reinterpret_cast<float4*>(sR + ((wave * RT + rt) * 64 + lane) * 4) =
            float4{acc[rt][0][0], acc[rt][0][1], acc[rt][0][2], acc[rt][0][3]};
      hc_sync();
      // value statistics of the rows (vpart; value_rows_kernel's per-row
      // terms, ppo.py:324-331), summed below in a fixed order
      double vs[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
      if (wave == 0 && li < a.out) {
        // one wait for the bias / target loads (and the HA2 copy-out stores
        // issued before them): without it the waitcnt pass, unsure of the bias
        // register across the row branches, waited vmcnt(0) in every row —
        // on the previous row's Y store
        __builtin_amdgcn_s_waitcnt(0x0F70);
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int r = 16 * rt + 4 * lk + i;
            if (r0 + r >= a.rows) continue;
            const float v = ((sR[((0 * RT + rt) * 64 + lane) * 4 + i] + sR[((1 * RT + rt) * 64 + lane) * 4 + i]) +
                             (sR[((2 * RT + rt) * 64 + lane) * 4 + i] + sR[((3 * RT + rt) * 64 + lane) * 4 + i])) + bn;
            const float y = a.tanh_out ? tanhf(v) : v;
            a.Y[(r0 + r) * a.ldy + li] = y;
            if (a.vgrad) {
              const float rv = vr[rt][i];
              a.vgrad[r0 + r] = a.vscale * (y - rv);
              if (a.vpart) {
                const float e = y - rv;
                const double dd = (double)rv - (double)y;
                vs[0] += (double)(e * e);
                vs[1] += dd; vs[2] += dd * dd;
                vs[3] += (double)rv; vs[4] += (double)rv * (double)rv;
              }
            }
            if constexpr (PS) smu[r * PA + li] = y;
          }
      }
      if (a.vpart && wave == 0) {        // lanes li >= out hold zeros
#pragma unroll
        for (int k = 0; k < 5; ++k) {
          const double t = wave_sum_d(vs[k]);
          if (lane == 0) a.vpart[(int64_t)blockIdx.x * 5 + k] = t;
        }
      }
    }
    if constexpr (PS) {
      // the statistics of the workgroup's rows (pol_rows.hpp: the stats
      // kernel's adapt-mode ops), summed over the rows on wave 0 in a fixed
      // butterfly order, one PS_N partial per workgroup
      hc_sync();
      double acc[PS_N];
#pragma unroll
      for (int k = 0; k < PS_N; ++k) acc[k] = 0.0;
      if (pown) {
        float sg[PA], lsg[PA], rsg[PA], mu[PA];
#pragma unroll
        for (int j = 0; j < PA; ++j) {
          sg[j] = expf(a.ps.lv[j]);                // builders.py:127 std = exp(log_var)
          lsg[j] = logf(sg[j]);
          rsg[j] = expf(a.ps.ref_lv[j]);
          mu[j] = smu[threadIdx.x * PA + j];
        }
        const PolStatsCols<PA> cols(sg, lsg, rsg, PA);
        const AdvNorm nadv(a.ps);
        pol_stats_row_adapt<PA>(a.ps, cols, nadv, mu, prm, pac, pbl, prbd, padv, pret, acc);
      }
      if (wave == 0) {
#pragma unroll
        for (int k = 0; k < PS_N; ++k) {
          const double v = wave_sum_d(acc[k]);
          if (lane == 0) a.ps.part[(int64_t)blockIdx.x * PS_N + k] = v;
        }
      }
    }
  }
  HEAD_TICK(0, 6);                                // HA2 copy-out + layer 3
  // side job for the backward of the same phase: W1^T, W2^T
  if (a.W1T) {
    const int t1 = ((a.h1 + 31) >> 5) * ((a.K0 + 31) >> 5);
    const int t2 = ((a.h2 + 31) >> 5) * ((a.h1 + 31) >> 5);
    for (int tix = blockIdx.x; tix < t1 + t2; tix += gridDim.x) {
      if (tix < t1) hc_transpose_tile(a.W1, a.h1, a.K0, a.W1T, tix, sR);
      else hc_transpose_tile(a.W2, a.h2, a.h1, a.W2T, tix - t1, sR);
    }
  }
  HEAD_TICK(0, 7);                                // transposes
  HEAD_END(0);
}

// PG: the policy loss gradient of the workgroup's rows as the prologue (the
// action width is the template's 8: out == 8)
template <int NTA, int NTB, int RT, bool PG>
__global__ void __launch_bounds__(kWG, RT == 1 ? 3 : 2)
head_bwd_kernel(HeadBwdArgs a) {
  if (a.skip && a.skip[0] != 0) return;
  constexpr int R = HC_R * RT;                    // rows per workgroup
  extern __shared__ __attribute__((aligned(16))) float hsm[];
  float* s2 = hsm;                                // [R][ld2]  dH2
  float* s1 = s2 + R * a.ld2;                     // [R][ld1]  dH1
  float* sZ = s1 + R * a.ld1;                     // [R][16]   dZ
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63, li = lane & 15, lk = lane >> 4;
  const int64_t r0 = (int64_t)blockIdx.x * R;
  const int out = a.out;
  HEAD_T0();
  // dZ rows (zero past out: the dH2 pass runs whole groups of 4 k), loaded
  // first; dH1's weight stream (W2^T) and its masks are issued behind them and
  // stay in flight through the dZ W3 pass
  const int zr = threadIdx.x >> 4, zk = threadIdx.x & 15;
  HcStream<NTA> SA;
  if constexpr (PG) {
    // thread t < R: row r0 + t's inputs, then the weight stream, then the
    // epoch's loss weights (and, one rank, its decision: every load above is
    // in flight meanwhile), then the row's dz and d/dstd terms (pol_rows.hpp,
    // the same ops as policy_rows_grad_kernel's row pass)
    constexpr int AT = 8;
    __shared__ PolGradShared psh;
    const int t = threadIdx.x;
    const int64_t n = r0 + t;
    const bool own = t < R && n < a.rows;
    PolGradRow<AT> x;
    if (own) x.load(a.pg, n, AT);
    SA.init(a.W2T, a.h2, a.h2, a.h1, wave, 4, 0, 1);
    float wsurr, wkl;
    PolGradPre pre;
    // one 64-partial slab per round trip: a deeper group of slabs in flight
    // pushed the one-row-tile forms into scratch spills (<5, 2, 1>: 143 -> 168
    // VGPRs + 80 B); a rank's 128 segments have 42 partials
    if (pol_grad_weights<1>(a.pg, psh, wsurr, wkl, pre)) return;
    const PolGradCols<AT> cols(pre, psh, AT);
    const AdvNorm nadv(a.pg, pre.mom);
    float glv[AT];
#pragma unroll
    for (int j = 0; j < AT; ++j) glv[j] = 0.f;
    if (t < R) {
      float dz[AT];
      if (own) {
        pol_grad_compute<AT>(a.pg, cols, nadv, x, wsurr, wkl, dz, glv);
        st_row<AT>(a.pg.dz + n * AT, dz, AT);
      } else {
#pragma unroll
        for (int j = 0; j < AT; ++j) dz[j] = 0.f;
      }
#pragma unroll
      for (int j = 0; j < 16; ++j) sZ[t * 16 + j] = j < AT ? dz[j] : 0.f;
    }
    if (wave == 0) {     // R <= 64: every row on wave 0; fixed butterfly order
#pragma unroll
      for (int j = 0; j < AT; ++j) {
        const float sg = wave_sum(glv[j]);
        if (lane == 0) a.pg.lvpart[(int64_t)blockIdx.x * AT + j] = sg;
      }
    }
  } else {
    float zv[RT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
      zv[rt] = a.dZ[min(r0 + 16 * rt + zr, a.rows - 1) * out + min(zk, out - 1)];
    SA.init(a.W2T, a.h2, a.h2, a.h1, wave, 4, 0, 1);
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) sZ[(16 * rt + zr) * 16 + zk] = zk < out ? zv[rt] : 0.f;
  }
  // padding columns of dH2 (the next layer's last chunk)
  const int h2p = a.ld2 - 4;
  for (int e = threadIdx.x; e < R * (h2p - a.h2); e += kWG) {
    const int r = e / (h2p - a.h2), c = e - r * (h2p - a.h2);
    s2[r * a.ld2 + a.h2 + c] = 0.f;
  }
  __syncthreads();
  // dH2 = (dZ W3) * [HA2 > 0], K = out: lane = a 4-column group, wave = 4
  // rows of each row tile; the k-ordered fmaf chain from 0 (steps k >= out add
  // 0 * w).  Per column pass, every W3 row group (out <= 16: <= 4 groups) and
  // the HA2 masks of all row tiles are loaded before the first FMA: one memory
  // round trip per pass instead of one per (row tile, k group) — the same FMAs
  // in the same order
  const int nq = a.h2 >> 2;              // <= 128: at most two passes, unrolled (a loop
#pragma unroll                           // header made the first pass drain every load
  for (int q0 = 0; q0 < 128; q0 += 64) {  // in flight, the weight prefetch included)
    if (q0 >= nq) break;
    const bool qv = q0 + lane < nq;
    const int q = qv ? q0 + lane : nq - 1;
    constexpr int KGM = 4;               // k groups of 4 (out <= 16)
    f32x4 w[KGM][4], m[RT][4];
#pragma unroll
    for (int g = 0; g < KGM; ++g)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        w[g][j] = *reinterpret_cast<const f32x4*>(a.W3 + (int64_t)min(4 * g + j, out - 1) * a.h2 + 4 * q);
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int64_t rr = min(r0 + 16 * rt + 4 * wave + i, a.rows - 1);
        m[rt][i] = *reinterpret_cast<const f32x4*>(a.HA2 + rr * a.h2 + 4 * q);
      }
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      f32x4 v[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int g = 0; g < KGM; ++g) {
        if (4 * g >= out) break;
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float z = sZ[(16 * rt + 4 * wave + i) * 16 + 4 * g + j];
            v[i][0] = fmaf(z, w[g][j][0], v[i][0]); v[i][1] = fmaf(z, w[g][j][1], v[i][1]);
            v[i][2] = fmaf(z, w[g][j][2], v[i][2]); v[i][3] = fmaf(z, w[g][j][3], v[i][3]);
          }
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = 16 * rt + 4 * wave + i;
        const f32x4 o = {m[rt][i][0] > 0.f ? v[i][0] : 0.f, m[rt][i][1] > 0.f ? v[i][1] : 0.f,
                         m[rt][i][2] > 0.f ? v[i][2] : 0.f, m[rt][i][3] > 0.f ? v[i][3] : 0.f};
        if (qv) {
          *reinterpret_cast<f32x4*>(s2 + r * a.ld2 + 4 * q) = o;
          if (r0 + r < a.rows) *reinterpret_cast<f32x4*>(a.dH2 + (r0 + r) * a.h2 + 4 * q) = o;
        }
      }
    }
  }
  // dH1's masks, in flight behind its k loop (issued here rather than with the
  // weight prefetch: fewer registers live through the dZ W3 pass)
  float eA[RT][NTA][4];
  hc_epi_load<NTA, 1, RT>(wave, a.h1, nullptr, a.HA1, r0, a.rows, eA);
  hc_sync();
  HEAD_TICK(1, 0);                                // dZ W3 pass
  HcStream<NTB> SB;
  {   // dH1 = (dH2 W2) * [HA1 > 0] = dH2 (W2^T)^T
    f32x4 acc[RT][NTA];
    hc_run<NTA, RT, true>(SA, s2, a.ld2, acc);
    HEAD_TICK(1, 1);                              // dH1 k loop
    if (a.dxn > 0)      // dX's weight stream (rows dx0.. of W1^T), in flight
      SB.init(a.W1T + (int64_t)a.dx0 * a.h1, a.h1, a.h1, a.dxn, wave, 4, 0, 1);
    hc_store<NTA, 1, RT>(acc, eA, wave, a.h1, s1, a.ld1);
  }
  hc_sync();
  HEAD_TICK(1, 2);                                // epilogue + barrier
  hc_copy_out<RT>(s1, a.ld1, a.h1, a.dH1, r0, a.rows);
  HEAD_TICK(1, 3);                                // dH1 copy-out issue
  if (a.dxn <= 0) { HEAD_END(1); return; }
  {   // dX = dH1 W1[:, dx0 : dx0 + dxn]
    f32x4 acc[RT][NTB];
    hc_run<NTB, RT, true>(SB, s1, a.ld1, acc);
    HEAD_TICK(1, 4);                              // dX k loop
    const int CT = (a.dxn + 15) >> 4;
#pragma unroll
    for (int t = 0; t < NTB; ++t) {
      const int nt = wave + 4 * t;
      if (nt >= CT) break;
      const int n = 16 * nt + li;
      if (n >= a.dxn) continue;
#pragma unroll
      for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int64_t r = r0 + 16 * rt + 4 * lk + i;
          if (r >= a.rows) continue;
          float v = acc[rt][t][i];
          if (a.mask) v = a.mask[r * a.ldm + n] > 0.f ? v : 0.f;
          a.dX[r * a.lddx + n] = v;
        }
    }
  }
  HEAD_TICK(1, 5);                                // dX epilogue
  HEAD_END(1);
}

#ifdef SMI_PROF
extern "C" int smi_head_phase_ticks(unsigned long long* out /* [2][10] */) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_head_ticks), sizeof(g_head_ticks)) != hipSuccess)
    return SMI_E_LAUNCH;
  static const unsigned long long zero[20] = {};
  return hipMemcpyToSymbol(HIP_SYMBOL(g_head_ticks), zero, sizeof(zero)) == hipSuccess ? SMI_OK
                                                                                        : SMI_E_LAUNCH;
}
#endif

// ------------------------------------------------------------------ host side
static int use_head_fused() {
  static int u = -1;
  if (u < 0) {
    const char* e = getenv("SMI_HEAD_FUSED");
    u = (e && e[0] == '0') ? 0 : 1;
  }
  return u;
}

static int hc_nt(int n) {                        // tiles per wave, rounded to an instantiation
  const int t = (((n + 15) >> 4) + 3) >> 2;
  return t <= 2 ? 2 : t <= 4 ? t : t <= 5 ? 5 : 8;     // 2, 3, 4, 5, 8
}

static bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

// shapes the fused chains take (the caller falls back to the layer GEMMs
// otherwise); the backward additionally needs dxn <= 320 (its dX tiles)
bool head_fused_ok(int in, int64_t ldx, int h1, int h2, int out, const float* X,
                   const float* W1, const float* W2, const float* W3) {
  return use_head_fused() && in >= 4 && in <= 320 && in % 4 == 0 && ldx % 4 == 0 &&
         h1 >= 4 && h1 <= HC_MAXK && h1 % 4 == 0 && h2 >= 4 && h2 <= HC_MAXK && h2 % 4 == 0 &&
         out >= 1 && out <= 16 && al16(X) && al16(W1) && al16(W2) && al16(W3);
}

// row tiles per workgroup: 2 (32 rows: the weight chunks feed twice the MFMAs)
// once the batch leaves at least ~2 workgroups per CU of them, else 1
// (SMI_HEAD_RT = 1 | 2 forces one: A/B knob)
static int hc_rt(int64_t rows) {
  static int force = -1;
  if (force < 0) {
    const char* e = getenv("SMI_HEAD_RT");
    force = e ? atoi(e) : 0;
    if (force != 1 && force != 2) force = 0;
  }
  if (force) return force;
  return rows >= 16384 ? 2 : 1;
}

// workgroups of a fused head launch over rows (the policy prologue writes one
// log_var partial per workgroup)
int head_bwd_blocks(int64_t rows) {
  const int R = HC_R * hc_rt(rows);
  return (int)((rows + R - 1) / R);
}

// the statistics epilogue's instantiation (C3 / C5 widths)
bool head_fwd_ps_ok(int h1, int h2, int out) { return hc_nt(h1) == 5 && hc_nt(h2) == 4 && out == 8; }

int launch_head_fwd_fused(const float* X, int64_t ldx, int64_t rows, int in, const float* W1,
                          const float* b1, int h1, const float* W2, const float* b2, int h2,
                          const float* W3, const float* b3, int out, int tanh_out, float* HA1,
                          float* HA2, float* Y, int64_t ldy, float* W1T, float* W2T,
                          hipStream_t st, const int* skip, const float* vret, float* vgrad,
                          float vscale, const PolRowArgs* ps, double* vpart) {
  if (rows <= 0) return SMI_OK;
  if (vgrad && (out != 1 || !vret)) return set_error(SMI_E_ARG, "head_forward: value epilogue needs out == 1");
  if (vpart && !vgrad) return set_error(SMI_E_ARG, "head_forward: value statistics need the value epilogue");
  if (ps && !head_fwd_ps_ok(h1, h2, out)) return set_error(SMI_E_ARG, "head_forward: statistics epilogue shape");
  HeadFwdArgs a{X, ldx, in, W1, b1, W2, b2, W3, b3, h1, h2, out, tanh_out, HA1, HA2, Y, ldy,
                W1T, W2T, rows, skip, hc_ld(in), hc_ld(h1), hc_ld(h2), vret, vgrad, vscale};
  if (ps) a.ps = *ps;
  a.vpart = vpart;
  const int rt = hc_rt(rows);
  const int R = HC_R * rt;
  const size_t lds = (size_t)(R * ((a.ld0 > a.ld2 ? a.ld0 : a.ld2) + a.ld1) + hc_sr(rt)) * 4;
  const dim3 grid((unsigned)((rows + R - 1) / R));
  const int n1 = hc_nt(h1), n2 = hc_nt(h2);
  const int kslot = ktime_begin(st);
#define SMI_HFP(A, B, P)                                                                \
  do {                                                                                  \
    if (rt == 2) {                                                                      \
      allow_lds(head_fwd_kernel<A, B, 2, P>, lds);                                      \
      hipLaunchKernelGGL((head_fwd_kernel<A, B, 2, P>), grid, dim3(kWG), lds, st, a);   \
    } else {                                                                            \
      allow_lds(head_fwd_kernel<A, B, 1, P>, lds);                                      \
      hipLaunchKernelGGL((head_fwd_kernel<A, B, 1, P>), grid, dim3(kWG), lds, st, a);   \
    }                                                                                   \
  } while (0)
#define SMI_HF(A, B) SMI_HFP(A, B, false)
  if (ps) {                        // the statistics epilogue: 300 x 200 heads, 8 actions
    SMI_HFP(5, 4, true);
    ktime_end(kslot, KT_GEMM_FWD,
              2.0 * (double)rows * ((double)in * h1 + (double)h1 * h2 + (double)h2 * out), st);
    return check_launch("head_fwd_kernel");
  }
  // layer-1 slots {2, 5, 8} x layer-2 slots {2, 3, 4, 5, 8} (C3 / C5: 300 x 200 -> 5, 4)
  const int m1 = n1 <= 2 ? 2 : n1 <= 5 ? 5 : 8;
#define SMI_HF2(A)                                        \
  do {                                                    \
    switch (n2) {                                         \
      case 2: SMI_HF(A, 2); break;                        \
      case 3: SMI_HF(A, 3); break;                        \
      case 4: SMI_HF(A, 4); break;                        \
      case 5: SMI_HF(A, 5); break;                        \
      default: SMI_HF(A, 8); break;                       \
    }                                                     \
  } while (0)
  if (m1 == 2) SMI_HF2(2);
  else if (m1 == 5) SMI_HF2(5);
  else SMI_HF2(8);
#undef SMI_HF2
#undef SMI_HF
#undef SMI_HFP
  ktime_end(kslot, KT_GEMM_FWD,
            2.0 * (double)rows * ((double)in * h1 + (double)h1 * h2 + (double)h2 * out), st);
  return check_launch("head_fwd_kernel");
}

int launch_head_bwd_fused(const float* dZ, int out, int64_t rows, const float* W3,
                          const float* W2T, const float* W1T, int h1, int h2, int dx0, int dxn,
                          const float* HA1, const float* HA2, float* dH2, float* dH1, float* dX,
                          int64_t lddx, const float* mask, int64_t ldm, hipStream_t st,
                          const int* skip, const PolRowArgs* pg) {
  if (rows <= 0) return SMI_OK;
  if (pg && out != 8) return set_error(SMI_E_ARG, "head_backward: the policy prologue needs out == 8");
  HeadBwdArgs a{dZ, out, W3, W2T, W1T, h1, h2, dx0, dxn, HA1, HA2, dH2, dH1, dX, lddx, mask, ldm,
                rows, skip, hc_ld(h2), hc_ld(h1)};
  if (pg) a.pg = *pg;
  const int rt = hc_rt(rows);
  const int R = HC_R * rt;
  const size_t lds = (size_t)(R * (a.ld2 + a.ld1) + R * 16) * 4;
  const dim3 grid((unsigned)((rows + R - 1) / R));
  int na = hc_nt(h1), nb = hc_nt(dxn > 0 ? dxn : 1);
  na = na <= 2 ? 2 : na <= 5 ? 5 : 8;
  nb = nb <= 2 ? 2 : 5;
  const int kslot = ktime_begin(st);
#define SMI_HB2(A, B, P)                                                               \
  do {                                                                                 \
    if (rt == 2) {                                                                     \
      allow_lds(head_bwd_kernel<A, B, 2, P>, lds);                                     \
      hipLaunchKernelGGL((head_bwd_kernel<A, B, 2, P>), grid, dim3(kWG), lds, st, a);  \
    } else {                                                                           \
      allow_lds(head_bwd_kernel<A, B, 1, P>, lds);                                     \
      hipLaunchKernelGGL((head_bwd_kernel<A, B, 1, P>), grid, dim3(kWG), lds, st, a);  \
    }                                                                                  \
  } while (0)
#define SMI_HB(A, B)                                                                   \
  do {                                                                                 \
    if (pg) SMI_HB2(A, B, true);                                                       \
    else SMI_HB2(A, B, false);                                                         \
  } while (0)
  if (na == 2 && nb == 2) SMI_HB(2, 2);
  else if (na == 2) SMI_HB(2, 5);
  else if (na == 5 && nb == 2) SMI_HB(5, 2);
  else if (na == 5) SMI_HB(5, 5);
  else if (nb == 2) SMI_HB(8, 2);
  else SMI_HB(8, 5);
#undef SMI_HB
#undef SMI_HB2
  ktime_end(kslot, KT_GEMM_DX,
            2.0 * (double)rows * ((double)out * h2 + (double)h2 * h1 + (double)h1 * dxn), st);
  return check_launch("head_bwd_kernel");
}

}  // namespace smi
