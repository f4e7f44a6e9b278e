// lstm_kernels.hip — the nn.LSTM stem of PPOModel (surreal/model/ppo_net.py:
// 137-152, 277-279, 310-312) as persistent sequence kernels for gfx950.
//
// The input projection x W_ih^T + b_ih of every step is one large GEMM
// (linear_kernels.hip) before the recurrence; what stays sequential is
//   gates_t = xproj_t + (h_{t-1} W_hh^T + b_hh)          [torch order i,f,g,o]
//   c_t = sigmoid(f) c_{t-1} + sigmoid(i) tanh(g),  h_t = sigmoid(o) tanh(c_t)
// Segments are independent, so one workgroup owns 16 segments for ALL steps
// (no inter-workgroup synchronisation): h_{t-1} lives in LDS as the MFMA A
// operand, c_{t-1} in registers, W_hh streams from L2 (160 KB at H = 100,
// shared by every workgroup).  Wave w owns hidden-unit tiles ut = w, w+4, ...
// of 16 units and computes the four gate columns of each (4 accumulators of
// v_mfma_f32_16x16x4_f32), so the cell update happens in the MFMA output
// registers: lane (li, lk) holds rows lk*4..lk*4+3 of unit ut*16+li.
//
// Backward (BPTT, reverse over steps) keeps dh_rec and dc in the same
// registers: dgates_t are formed element-wise, written to HBM (for the weight
// GEMMs) and to LDS, and dh_rec_{t-1} = dgates_t W_hh is the next MFMA pass
// (K = 4H, B operand contiguous along units).
#include <stdlib.h>
#include "smi_device.hpp"
#include "smi_internal.hpp"
#include "lstm_cell.hpp"

// The file is compiled twice (build.py): SMI_LSTM_PART 1 = the MFMA forms and
// the launchers, SMI_LSTM_PART 2 = the VALU recurrence (lstm_fwd_v_kernel /
// lstm_bwd_v_kernel) with -fno-slp-vectorize.  The VALU recurrence's fmaf
// chains must stay scalar v_fmac_f32 (the SLP vectorizer packs them into
// v_pk_fma_f32 + operand moves: same sums, slower); the flag on the MFMA forms
// changed their rounding, so it is applied to the VALU half only.
// 0 (default) = both halves in one object.
#ifndef SMI_LSTM_PART
#define SMI_LSTM_PART 0
#endif
#define SMI_LSTM_MFMA (SMI_LSTM_PART != 2)
#define SMI_LSTM_VALU_HALF (SMI_LSTM_PART != 1)

namespace smi {

[[maybe_unused]] constexpr int LR = 16;   // segments per workgroup

// Developer phase timer (build variant 'prof', -DSMI_PROF): workgroup 0, wave
// 0 accumulates wall-clock ticks (100 MHz) per step phase:
//   [0] fwd MFMA (incl. LDS operand reads)  [1] fwd epilogue  [2] fwd barrier
//   [3] bwd element-wise + stores           [4] bwd barrier   [5] bwd MFMA
#ifdef SMI_PROF
__device__ unsigned long long g_lstm_ticks[8];
#define LSTM_T0() unsigned long long t_prev_ = wall_clock64()
#define LSTM_TICK(id)                                                       \
  do {                                                                      \
    if (blockIdx.x == 0 && threadIdx.x == 0) {                              \
      const unsigned long long n_ = wall_clock64();                         \
      g_lstm_ticks[id] += n_ - t_prev_;                                     \
      t_prev_ = n_;                                                         \
    }                                                                       \
  } while (0)
#else
#define LSTM_T0() (void)0
#define LSTM_TICK(id) (void)0
#endif

// LDS leading dim for a [16][K] A-operand image: >= round4(K) and == 4 (mod 8),
// so the 16 rows x 4 k of one MFMA operand read hit 64 distinct banks.
__host__ __device__ inline int lstm_ld(int k) {
  int l = round4(k);
  if ((l & 7) != 4) l += 4;
  return l;
}

// Activations (sigm, ftanh): lstm_cell.hpp.
// k-order of the register kernels: lane group lk (= lane >> 4) owns the
// contiguous quarter k = lk*KS + s, s < KS, of the (padded) K range, so the A
// operand of 4 consecutive k-steps is one 16-byte LDS read (the MFMA only needs
// every k to appear once across the 4 lane groups).
__host__ __device__ inline int lstm_q(int K) { return (((K + 3) >> 2) + 3) & ~3; }

#if SMI_LSTM_MFMA
template <int MAXUT>
__global__ void __launch_bounds__(kWG)
lstm_fwd_kernel(LstmFwdArgs a) {
  if (a.skip && a.skip[0] != 0) return;
  const int keepS = a.keep > 0 ? a.keep : a.S;     // steps whose c / gates are stored
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int H = a.H, B = a.B, G4 = 4 * H;
  const int LDH = lstm_ld(4 * lstm_q(H));
  float* hA[2] = {sm, sm + LR * LDH};
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int li = lane & 15, lk = lane >> 4;
  const int r0 = blockIdx.x * LR;
  const int NUT = (H + 15) >> 4;
  const int64_t BH = (int64_t)B * H;
  for (int e = threadIdx.x; e < LR * LDH; e += kWG) {
    const int r = e / LDH, k = e - r * LDH;
    const bool ok = k < H && r0 + r < B;
    const float v = ok ? a.h0[(int64_t)(r0 + r) * H + k] : 0.f;
    hA[0][e] = v;
    hA[1][e] = 0.f;
    if (ok) a.hbuf[(int64_t)(r0 + r) * H + k] = v;        // hbuf[0] = h0
  }
  float creg[MAXUT][4];
#pragma unroll
  for (int u = 0; u < MAXUT; ++u) {
    const int unit = (wave + 4 * u) * 16 + li;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int gr = r0 + lk * 4 + i;
      const bool ok = unit < H && gr < B;
      creg[u][i] = ok ? a.c0[(int64_t)gr * H + unit] : 0.f;
      if (ok && a.cbuf) a.cbuf[(int64_t)gr * H + unit] = creg[u][i];
    }
  }
  // per-lane W_hh row bases (clamped: rows of units >= H read unit H-1 and are
  // never stored)
  const float* wrow[MAXUT][4];
  float bh[MAXUT][4];
#pragma unroll
  for (int u = 0; u < MAXUT; ++u) {
    int unit = (wave + 4 * u) * 16 + li;
    unit = unit < H ? unit : H - 1;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      wrow[u][g] = a.w_hh + (int64_t)(g * H + unit) * H;
      bh[u][g] = a.b_hh[g * H + unit];
    }
  }
  const int nks = (H + 3) >> 2;        // k-steps of 4
  __syncthreads();
  for (int t = 0; t < a.S; ++t) {
    const float* hp = hA[t & 1];
    float* hn = hA[(t + 1) & 1];
    // x-projection of this step (epilogue operand), issued before the MFMAs
    float xp[MAXUT][4][4];
#pragma unroll
    for (int u = 0; u < MAXUT; ++u) {
      int unit = (wave + 4 * u) * 16 + li;
      unit = unit < H ? unit : H - 1;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        int gr = r0 + lk * 4 + i;
        gr = gr < B ? gr : B - 1;
        const float* xr = a.xproj + ((int64_t)t * B + gr) * G4 + unit;
#pragma unroll
        for (int g = 0; g < 4; ++g) xp[u][g][i] = xr[g * H];
      }
    }
    f32x4 acc[MAXUT][4];
#pragma unroll
    for (int u = 0; u < MAXUT; ++u)
#pragma unroll
      for (int g = 0; g < 4; ++g) acc[u][g] = f32x4{0.f, 0.f, 0.f, 0.f};
    const float* ap = hp + li * LDH + lk;
    int ks = 0;
    for (; ks + 4 <= nks; ks += 4) {
      float av[4], bv[MAXUT][4][4];
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int k = (ks + s) * 4 + lk;
        const int kc = k < H ? k : H - 1;         // A is zero there (LDS pad)
        av[s] = ap[(ks + s) * 4];
#pragma unroll
        for (int u = 0; u < MAXUT; ++u)
#pragma unroll
          for (int g = 0; g < 4; ++g) bv[u][g][s] = wrow[u][g][kc];
      }
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int u = 0; u < MAXUT; ++u)
#pragma unroll
          for (int g = 0; g < 4; ++g) acc[u][g] = mfma4(av[s], bv[u][g][s], acc[u][g]);
    }
    for (; ks < nks; ++ks) {
      const int k = ks * 4 + lk;
      const int kc = k < H ? k : H - 1;
      const float av = ap[ks * 4];
#pragma unroll
      for (int u = 0; u < MAXUT; ++u)
#pragma unroll
        for (int g = 0; g < 4; ++g) acc[u][g] = mfma4(av, wrow[u][g][kc], acc[u][g]);
    }
    // cell update in the accumulator registers
#pragma unroll
    for (int u = 0; u < MAXUT; ++u) {
      const int ut = wave + 4 * u;
      const int unit = ut * 16 + li;
      if (ut >= NUT) continue;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = lk * 4 + i, gr = r0 + row;
        const float gi = xp[u][0][i] + (acc[u][0][i] + bh[u][0]);
        const float gf = xp[u][1][i] + (acc[u][1][i] + bh[u][1]);
        const float gg = xp[u][2][i] + (acc[u][2][i] + bh[u][2]);
        const float go = xp[u][3][i] + (acc[u][3][i] + bh[u][3]);
        const float ig = sigm(gi), fg = sigm(gf), cg = ftanh(gg), og = sigm(go);
        const float c = fg * creg[u][i] + ig * cg;
        const float h = og * ftanh(c);
        const bool ok = unit < H && gr < B;
        creg[u][i] = ok ? c : 0.f;
        if (unit < H) hn[row * LDH + unit] = ok ? h : 0.f;
        if (ok) {
          a.hbuf[(int64_t)(t + 1) * BH + (int64_t)gr * H + unit] = h;
          if (a.cbuf && t < keepS) a.cbuf[(int64_t)(t + 1) * BH + (int64_t)gr * H + unit] = c;
          if (a.gates && t < keepS) {
            float* gp = a.gates + ((int64_t)t * B + gr) * G4 + unit;
            gp[0] = ig; gp[H] = fg; gp[2 * H] = cg; gp[3 * H] = og;
          }
        }
      }
    }
    __syncthreads();
  }
}



template <int MAXUT>
__global__ void __launch_bounds__(kWG)
lstm_bwd_kernel(LstmBwdArgs a) {
  if (a.skip && a.skip[0] != 0) return;
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int H = a.H, B = a.B, G4 = 4 * H;
  const int LDG = lstm_ld(G4);
  float* dG[2] = {sm, sm + LR * LDG};
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int li = lane & 15, lk = lane >> 4;
  const int r0 = blockIdx.x * LR;
  const int NUT = (H + 15) >> 4;
  const int64_t BH = (int64_t)B * H;
  for (int e = threadIdx.x; e < 2 * LR * LDG; e += kWG) sm[e] = 0.f;
  float dcreg[MAXUT][4];
  f32x4 dhrec[MAXUT];
#pragma unroll
  for (int u = 0; u < MAXUT; ++u) {
    dhrec[u] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 4; ++i) dcreg[u][i] = 0.f;
  }
  int ucl[MAXUT];
#pragma unroll
  for (int u = 0; u < MAXUT; ++u) {
    const int unit = (wave + 4 * u) * 16 + li;
    ucl[u] = unit < H ? unit : H - 1;
  }
  const int nks = G4 >> 2;              // K = 4H, k-steps of 4
  __syncthreads();
  for (int t = a.S - 1; t >= 0; --t) {
    float* dg = dG[t & 1];
#pragma unroll
    for (int u = 0; u < MAXUT; ++u) {
      const int ut = wave + 4 * u;
      const int unit = ut * 16 + li;
      if (ut >= NUT) continue;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = lk * 4 + i;
        int gr = r0 + row;
        const bool ok = unit < H && gr < B;
        gr = gr < B ? gr : B - 1;
        const int uc = ucl[u];
        const float* gp = a.gates + ((int64_t)t * B + gr) * G4 + uc;
        const float ig = gp[0], fg = gp[H], cg = gp[2 * H], og = gp[3 * H];
        const float c = a.cbuf[(int64_t)(t + 1) * BH + (int64_t)gr * H + uc];
        const float cp = a.cbuf[(int64_t)t * BH + (int64_t)gr * H + uc];
        const float dh = a.dh[(int64_t)t * BH + (int64_t)gr * H + uc] + dhrec[u][i];
        const float tc = ftanh(c);
        const float dc = dh * og * (1.f - tc * tc) + dcreg[u][i];
        const float d_o = (dh * tc) * (og * (1.f - og));
        const float d_i = (dc * cg) * (ig * (1.f - ig));
        const float d_g = (dc * ig) * (1.f - cg * cg);
        const float d_f = (dc * cp) * (fg * (1.f - fg));
        dcreg[u][i] = ok ? dc * fg : 0.f;
        if (ok) {
          float* o = a.dgates + ((int64_t)t * B + gr) * G4 + unit;
          o[0] = d_i; o[H] = d_f; o[2 * H] = d_g; o[3 * H] = d_o;
          float* l = dg + row * LDG + unit;
          l[0] = d_i; l[H] = d_f; l[2 * H] = d_g; l[3 * H] = d_o;
        }
      }
    }
    __syncthreads();
    if (t == 0) break;
    // dh_rec for step t-1:  dgates_t (16 x 4H) @ W_hh (4H x H)
#pragma unroll
    for (int u = 0; u < MAXUT; ++u) dhrec[u] = f32x4{0.f, 0.f, 0.f, 0.f};
    const float* ap = dg + li * LDG + lk;
    int ks = 0;
    for (; ks + 8 <= nks; ks += 8) {
      float av[8], bv[MAXUT][8];
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        const int k = (ks + s) * 4 + lk;
        av[s] = ap[(ks + s) * 4];
#pragma unroll
        for (int u = 0; u < MAXUT; ++u) bv[u][s] = a.w_hh[(int64_t)k * H + ucl[u]];
      }
#pragma unroll
      for (int s = 0; s < 8; ++s)
#pragma unroll
        for (int u = 0; u < MAXUT; ++u) dhrec[u] = mfma4(av[s], bv[u][s], dhrec[u]);
    }
    for (; ks < nks; ++ks) {
      const int k = ks * 4 + lk;
      const float av = ap[ks * 4];
#pragma unroll
      for (int u = 0; u < MAXUT; ++u) dhrec[u] = mfma4(av, a.w_hh[(int64_t)k * H + ucl[u]], dhrec[u]);
    }
  }
}

// ---------------------------------------------------------------------------
// Register-resident variants (H <= 100, the reference's default H = 100): 8
// waves, wave w owns unit tile w, and its slice of W_hh (4 gates x 16 units x
// H for the forward; 16 units x 4H for the backward) is loaded ONCE into
// registers — every step then runs at the MFMA rate with one LDS read per
// k-step (the h_{t-1} / dgates operand) instead of streaming 160 KB of W_hh
// from L2 per step.  KS = k-steps of 4 held per lane (compile-time bound;
// steps past the runtime count are uniform-branch skipped).
constexpr int kWG8 = 512;

template <int KS>
__global__ void __launch_bounds__(kWG8)
lstm_fwd_reg_kernel(LstmFwdArgs a) {
  if (a.skip && a.skip[0] != 0) return;
  const int keepS = a.keep > 0 ? a.keep : a.S;     // steps whose c / gates are stored
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int H = a.H, B = a.B, G4 = 4 * H;
  const int LDH = lstm_ld(4 * KS);
  float* hA[2] = {sm, sm + LR * LDH};
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int li = lane & 15, lk = lane >> 4;
  const int r0 = blockIdx.x * LR;
  const int NUT = (H + 15) >> 4;
  const int64_t BH = (int64_t)B * H;
  const bool active = wave < NUT;
  const int unit = wave * 16 + li;
  const int uc = unit < H ? unit : H - 1;
  for (int e = threadIdx.x; e < LR * LDH; e += kWG8) {
    const int r = e / LDH, k = e - r * LDH;
    const bool ok = k < H && r0 + r < B;
    const float v = ok ? a.h0[(int64_t)(r0 + r) * H + k] : 0.f;
    hA[0][e] = v;
    hA[1][e] = 0.f;
    if (ok) a.hbuf[(int64_t)(r0 + r) * H + k] = v;        // hbuf[0] = h0
  }
  float w[4][KS];
  float bh[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const float* wr = a.w_hh + (int64_t)(g * H + uc) * H;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int k = lk * KS + s;
      const float x = wr[k < H ? k : H - 1];
      w[g][s] = k < H ? x : 0.f;
    }
    bh[g] = a.b_hh[g * H + uc];
  }
  float creg[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int gr = r0 + lk * 4 + i;
    const bool ok = active && unit < H && gr < B;
    creg[i] = ok ? a.c0[(int64_t)gr * H + unit] : 0.f;
    if (ok && a.cbuf) a.cbuf[(int64_t)gr * H + unit] = creg[i];
  }
  __syncthreads();
  LSTM_T0();
  for (int t = 0; t < a.S; ++t) {
    const float* hp = hA[t & 1];
    float* hn = hA[(t + 1) & 1];
    if (active) {
      float xp[4][4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        int gr = r0 + lk * 4 + i;
        gr = gr < B ? gr : B - 1;
        const float* xr = a.xproj + ((int64_t)t * B + gr) * G4 + uc;
#pragma unroll
        for (int g = 0; g < 4; ++g) xp[g][i] = xr[g * H];
      }
      f32x4 acc[4];
#pragma unroll
      for (int g = 0; g < 4; ++g) acc[g] = f32x4{0.f, 0.f, 0.f, 0.f};
      const float4* ap4 = reinterpret_cast<const float4*>(hp + li * LDH + lk * KS);
#pragma unroll
      for (int s4 = 0; s4 < KS / 4; ++s4) {
        const float4 av = ap4[s4];
        const float avs[4] = {av.x, av.y, av.z, av.w};
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int g = 0; g < 4; ++g) acc[g] = mfma4(avs[j], w[g][4 * s4 + j], acc[g]);
      }
      LSTM_TICK(0);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = lk * 4 + i, gr = r0 + row;
        const float gi = xp[0][i] + (acc[0][i] + bh[0]);
        const float gf = xp[1][i] + (acc[1][i] + bh[1]);
        const float gg = xp[2][i] + (acc[2][i] + bh[2]);
        const float go = xp[3][i] + (acc[3][i] + bh[3]);
        const float ig = sigm(gi), fg = sigm(gf), cg = ftanh(gg), og = sigm(go);
        const float c = fg * creg[i] + ig * cg;
        const float h = og * ftanh(c);
        const bool ok = unit < H && gr < B;
        creg[i] = ok ? c : 0.f;
        if (unit < H) hn[row * LDH + unit] = ok ? h : 0.f;
        if (ok) {
          a.hbuf[(int64_t)(t + 1) * BH + (int64_t)gr * H + unit] = h;
          if (a.cbuf && t < keepS) a.cbuf[(int64_t)(t + 1) * BH + (int64_t)gr * H + unit] = c;
          if (a.gates && t < keepS) {
            float* gp = a.gates + ((int64_t)t * B + gr) * G4 + unit;
            gp[0] = ig; gp[H] = fg; gp[2 * H] = cg; gp[3 * H] = og;
          }
        }
      }
      LSTM_TICK(1);
    }
    __syncthreads();
    LSTM_TICK(2);
  }
}

template <int KS>
__global__ void __launch_bounds__(kWG8)
lstm_bwd_reg_kernel(LstmBwdArgs a) {
  if (a.skip && a.skip[0] != 0) return;
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int H = a.H, B = a.B, G4 = 4 * H;
  const int LDG = lstm_ld(G4);
  float* dG[2] = {sm, sm + LR * LDG};
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int li = lane & 15, lk = lane >> 4;
  const int r0 = blockIdx.x * LR;
  const int NUT = (H + 15) >> 4;
  const int64_t BH = (int64_t)B * H;
  const bool active = wave < NUT;
  const int unit = wave * 16 + li;
  const int uc = unit < H ? unit : H - 1;
  for (int e = threadIdx.x; e < 2 * LR * LDG; e += kWG8) sm[e] = 0.f;
  float w[KS];                          // W_hh[lk*KS + s][unit]  (KS == H, K = 4H)
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int k = lk * KS + s;
    w[s] = a.w_hh[(int64_t)(k < G4 ? k : G4 - 1) * H + uc];
  }
  // per-lane element offsets of the 4 rows (clamped rows read row B-1)
  int64_t roff[4];
  bool rok[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int gr = r0 + lk * 4 + i;
    rok[i] = unit < H && gr < B;
    roff[i] = (int64_t)(gr < B ? gr : B - 1);
  }
  // step operands, prefetched one step ahead (issued before the dh_rec MFMAs)
  float pg[4][4], pc[4], pcp[4], pdh[4];
  auto fetch = [&](int t) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float* gp = a.gates + ((int64_t)t * B + roff[i]) * G4 + uc;
      pg[i][0] = gp[0]; pg[i][1] = gp[H]; pg[i][2] = gp[2 * H]; pg[i][3] = gp[3 * H];
      pc[i] = a.cbuf[(int64_t)(t + 1) * BH + roff[i] * H + uc];
      pcp[i] = a.cbuf[(int64_t)t * BH + roff[i] * H + uc];
      pdh[i] = a.dh[(int64_t)t * BH + roff[i] * H + uc];
    }
  };
  if (active && a.S > 0) fetch(a.S - 1);
  float dcreg[4] = {0.f, 0.f, 0.f, 0.f};
  f32x4 dhrec = f32x4{0.f, 0.f, 0.f, 0.f};
  __syncthreads();
  LSTM_T0();
  for (int t = a.S - 1; t >= 0; --t) {
    float* dg = dG[t & 1];
    if (active) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = lk * 4 + i;
        const float ig = pg[i][0], fg = pg[i][1], cg = pg[i][2], og = pg[i][3];
        const float c = pc[i], cp = pcp[i];
        const float dh = pdh[i] + dhrec[i];
        const float tc = ftanh(c);
        const float dc = dh * og * (1.f - tc * tc) + dcreg[i];
        const float d_o = (dh * tc) * (og * (1.f - og));
        const float d_i = (dc * cg) * (ig * (1.f - ig));
        const float d_g = (dc * ig) * (1.f - cg * cg);
        const float d_f = (dc * cp) * (fg * (1.f - fg));
        dcreg[i] = rok[i] ? dc * fg : 0.f;
        if (rok[i]) {
          float* o = a.dgates + ((int64_t)t * B + roff[i]) * G4 + unit;
          o[0] = d_i; o[H] = d_f; o[2 * H] = d_g; o[3 * H] = d_o;
          float* l = dg + row * LDG + unit;
          l[0] = d_i; l[H] = d_f; l[2 * H] = d_g; l[3 * H] = d_o;
        }
      }
    }
    LSTM_TICK(3);
    __syncthreads();
    LSTM_TICK(4);
    if (t == 0) break;
    if (active) {
      fetch(t - 1);
      // two accumulator chains (alternating 4-step groups), 16-byte A reads
      f32x4 h0 = f32x4{0.f, 0.f, 0.f, 0.f}, h1 = f32x4{0.f, 0.f, 0.f, 0.f};
      const float4* ap4 = reinterpret_cast<const float4*>(dg + li * LDG + lk * KS);
#pragma unroll
      for (int s4 = 0; s4 < KS / 4; ++s4) {
        const float4 av = ap4[s4];
        if (s4 & 1) {
          h1 = mfma4(av.x, w[4 * s4], h1); h1 = mfma4(av.y, w[4 * s4 + 1], h1);
          h1 = mfma4(av.z, w[4 * s4 + 2], h1); h1 = mfma4(av.w, w[4 * s4 + 3], h1);
        } else {
          h0 = mfma4(av.x, w[4 * s4], h0); h0 = mfma4(av.y, w[4 * s4 + 1], h0);
          h0 = mfma4(av.z, w[4 * s4 + 2], h0); h0 = mfma4(av.w, w[4 * s4 + 3], h0);
        }
      }
      dhrec = h0 + h1;
      LSTM_TICK(5);
    }
  }
}

// ---------------------------------------------------------------------------
// 4-segment variants (H <= 128, the reference default H = 100 included): a
// workgroup owns LR4 = 4 segments, so the 1024-segment C3 batch spreads over
// 256 workgroups — one per CU — instead of 64.  A step's recurrent GEMM is
// then 4 rows x 4H columns x H, which is exactly the shape of
// v_mfma_f32_4x4x1_16b_f32 with block 0's A operand (the 4 rows of h_{t-1},
// lanes 0-3) broadcast to all 16 blocks (cbsz 4): a 4 x 64 outer-product
// step whose output column is the lane.  Wave w owns gate columns
// 64w .. 64w+63 with its W_hh column in registers; 8 accumulators over
// k mod 8 hide the 44-cycle dependent latency (measured: 12 cycles/MFMA at 4
// chains, tools/exp/mfma4x4.hip).  The cell update runs one (row, unit) per
// thread after the pre-activations pass through LDS.
//
// Backward: dh_rec = dgates_t (4 x 4H) W_hh (4H x H) with units on lanes
// (ceil(H/64) groups of 64) and K = 4H split over the waves of a group; the
// partial sums meet in LDS and are added in a fixed order by the cell threads.
// dst[k] = r[k] for k < n, 0 for n <= k < N: float4 runs when r is 16-byte
// aligned and n % 4 == 0, float2 runs when 8-byte aligned and n even, else
// scalar loads (the branch is uniform across a launch's rows when the row
// stride keeps the alignment)
template <int N>
__device__ __forceinline__ void load_row(const float* r, int n, float* dst) {
  static_assert(N % 4 == 0, "rows in float4 runs");
  const uintptr_t ad = reinterpret_cast<uintptr_t>(r);
  if ((ad & 15) == 0 && (n & 3) == 0) {
#pragma unroll
    for (int k = 0; k < N; k += 4) {
      const float4 v = k < n ? *reinterpret_cast<const float4*>(r + k) : float4{0.f, 0.f, 0.f, 0.f};
      dst[k] = v.x; dst[k + 1] = v.y; dst[k + 2] = v.z; dst[k + 3] = v.w;
    }
  } else if ((ad & 7) == 0 && (n & 1) == 0) {
#pragma unroll
    for (int k = 0; k < N; k += 2) {
      const float2 v = k < n ? *reinterpret_cast<const float2*>(r + k) : float2{0.f, 0.f};
      dst[k] = v.x; dst[k + 1] = v.y;
    }
  } else {
#pragma unroll
    for (int k = 0; k < N; ++k) dst[k] = k < n ? r[k] : 0.f;
  }
}

constexpr int LR4 = 4;
#ifndef SMI_LSTM_HQ
#define SMI_LSTM_HQ 4
#endif
constexpr int LSTM_HQ = SMI_LSTM_HQ;    // h float4 LDS reads in flight (forward r4)

__device__ __forceinline__ f32x4 mfma4x64(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c, 4, 0, 0);
}

// KP: H rounded up to a multiple of 8 (W_hh registers per lane).  KX > 0:
// the input projection is fused (din <= KX, a multiple of 8): W_ih's column
// joins W_hh's in registers, x_t of the 4 segments is staged in LDS one step
// ahead, and the k loop runs over [x_t | h_{t-1}] — no xproj GEMM and no
// [S][B][4H] round trip through HBM.
// r4 forward weight staging (round 6).  A lane's W_hh / W_ih row loaded
// straight from global memory puts 64 rows -- 64 cache lines -- behind every
// load instruction of the wave (the prologue: 11 us of a 54 us launch at C3,
// tools/lstm_ticks.py, tick 6).  Staged (A/B knob SMI_R4_WSTAGE=1, measured
// slower: 18.8 us), each pass
// is a contiguous block of rows read as float4 runs by the whole workgroup
// (R4_PT per thread, one trip), stored to LDS, and each lane then reads its
// own row from LDS; the next pass's global loads are in flight meanwhile.
constexpr int R4_PT = 11;
template <int N>
__device__ __forceinline__ void r4_row_from_lds(const float* lds, int rb, int rc, int len, int myrow,
                                                float (&dst)[N]) {
  if (myrow >= rb && myrow < rb + rc) {
    const float* r = lds + (myrow - rb) * len;
#pragma unroll
    for (int k = 0; k < N; ++k) {
      const float t = r[min(k, len - 1)];
      dst[k] = k < len ? t : 0.f;
    }
  }
}

// VF (round 6): the launcher checked that W_hh rows are float4 runs (H % 4 == 0,
// 16-byte aligned) and W_ih rows float2 runs (din even, 8-byte aligned), so the
// row loads take ONE vector width without a run-time branch -- load_row's
// uniform alignment branch made the waitcnt pass wait vmcnt(0) at its merge,
// serializing the W_hh and W_ih loads into separate memory round trips
// (n % V == 0: a run is wholly inside the row or wholly past it; runs past it
// read a zero vector by address -- a select on the loaded value would make
// the waitcnt pass wait for the load right there)
__device__ __attribute__((aligned(16))) float g_lstm_zero4[4] = {0.f, 0.f, 0.f, 0.f};
template <int N, int V>
__device__ __forceinline__ void load_row_v(const float* r, int n, float* dst) {
  static_assert(N % 4 == 0 && (V == 4 || V == 2), "vector rows");
#pragma unroll
  for (int k = 0; k < N; k += V) {
    const float* src = k < n ? r + k : g_lstm_zero4;
    if constexpr (V == 4) {
      const float4 v = *reinterpret_cast<const float4*>(src);
      dst[k] = v.x; dst[k + 1] = v.y; dst[k + 2] = v.z; dst[k + 3] = v.w;
    } else {
      const float2 v = *reinterpret_cast<const float2*>(src);
      dst[k] = v.x; dst[k + 1] = v.y;
    }
  }
}

template <int KP, int KX, bool VF = false>
__global__ void __launch_bounds__(kWG8)
lstm_fwd_r4_kernel(LstmFwdArgs a) {
  if (a.skip && a.skip[0] != 0) return;
  LSTM_T0();
  const int keepS = a.keep > 0 ? a.keep : a.S;     // steps whose c / gates are stored
  constexpr int KXS = KX > 0 ? KX : 8;
  __shared__ __attribute__((aligned(16))) float hS[2][LR4 * KP];
  __shared__ __attribute__((aligned(16))) float xS[2][LR4 * KXS];
  __shared__ float pre[LR4][4 * KP];
  const int H = a.H, B = a.B, G4 = 4 * H;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r0 = blockIdx.x * LR4;
  const int64_t BH = (int64_t)B * H;
  const int col = wave * 64 + lane;
  const bool cact = wave * 64 < G4;              // wave-uniform
  const int colc = col < G4 ? col : G4 - 1;
  float w[KP];
  float wx[KXS];
  float bh = a.b_hh[colc];
  if constexpr (KX > 0) bh += a.b_ih[colc];
  if (a.wstage) {                                  // (uniform; the launcher sized the LDS)
    extern __shared__ __attribute__((aligned(16))) float4 wst4[];
    const float* wst = reinterpret_cast<const float*>(wst4);
    float4 v[R4_PT];
    auto gload = [&](const float* M, int n4) {
#pragma unroll
      for (int j = 0; j < R4_PT; ++j)
        v[j] = reinterpret_cast<const float4*>(M)[min(tid + j * kWG8, n4 - 1)];
    };
    auto lstore = [&](int n4) {
#pragma unroll
      for (int j = 0; j < R4_PT; ++j) wst4[min(tid + j * kWG8, n4 - 1)] = v[j];
    };
    const int nh4 = (2 * H * H) >> 2;              // half of W_hh: rows [0, 2H) / [2H, 4H)
    if constexpr (KX > 0) {
      gload(a.w_ih, (G4 * a.din) >> 2);
      lstore((G4 * a.din) >> 2);
      __syncthreads();
      gload(a.w_hh, nh4);
      r4_row_from_lds<KX>(wst, 0, G4, a.din, colc, wx);
      __syncthreads();
    } else {
      gload(a.w_hh, nh4);
    }
    lstore(nh4);
    __syncthreads();
    gload(a.w_hh + (int64_t)2 * H * H, nh4);
    r4_row_from_lds<KP>(wst, 0, 2 * H, H, colc, w);
    __syncthreads();
    lstore(nh4);
    __syncthreads();
    r4_row_from_lds<KP>(wst, 2 * H, 2 * H, H, colc, w);
  } else {
    // the lane's W_hh (and W_ih) row in registers, loaded in 16- (8-) byte runs
    // where the rows allow (a load per k put 64 rows' lines behind every
    // instruction, 32 instructions per line)
    if constexpr (VF) {
      load_row_v<KP, 4>(a.w_hh + (int64_t)colc * H, H, w);
      if constexpr (KX > 0) load_row_v<KX, 2>(a.w_ih + (int64_t)colc * a.din, a.din, wx);
    } else {
      load_row<KP>(a.w_hh + (int64_t)colc * H, H, w);
      if constexpr (KX > 0) load_row<KX>(a.w_ih + (int64_t)colc * a.din, a.din, wx);
    }
  }
  // x staging: thread tid < 4*KX owns (row tid / KX, k tid % KX) of x_t
  const int xr = tid / KXS, xk = tid - (tid / KXS) * KXS;
  const bool xown = KX > 0 && tid < LR4 * KXS;
  const int64_t xoff0 = (int64_t)min(r0 + xr, B - 1) * a.ldx + min(xk, a.din - 1);
  const bool xval = xk < a.din;
  // the raw value (clamped address): the zero for k >= din is selected when it
  // is written to LDS a step later, so the load stays in flight across the
  // step (a select right after the load made the compiler wait vmcnt(0) on it
  // in every step, the x fetch latency on the recurrence's critical path)
  auto xload = [&](int t) -> float { return a.x[(int64_t)t * B * a.ldx + xoff0]; };
  // Round 6: x_0, x_1, c0 and h0 are loaded unconditionally (clamped
  // addresses, the selects after the loads) together with the weights above
  // and stored after; a load used only under a per-lane condition (xown, ok)
  // was sunk into that branch and waited on there, one round trip each
  float xnext = 0.f, x0 = 0.f;
  if constexpr (KX > 0) {
    x0 = xload(0);
    xnext = xload(a.S > 1 ? 1 : 0);
  }
  // cell owned by this thread: (crow, cunit)
  const bool cell = tid < LR4 * H;
  const int crow = cell ? tid / H : 0;
  const int cunit = cell ? tid - crow * H : 0;
  const int cgr = r0 + crow;
  const bool cok = cell && cgr < B;
  const float c0v = a.c0[(int64_t)min(cgr, B - 1) * H + cunit];
  static_assert(LR4 * KP <= kWG8, "one h0 slot per thread");
  const int he = min(tid, LR4 * KP - 1);
  const int hr = he / KP, hk = he - hr * KP;
  float h0v = a.h0[(int64_t)min(r0 + hr, B - 1) * H + min(hk, H - 1)];
  // (pinned: their only uses sit under per-lane conditions)
  asm volatile("" : "+v"(h0v));
  if constexpr (KX > 0) asm volatile("" : "+v"(x0));
  if constexpr (KX > 0) {
    if (xown && a.S > 0) xS[0][xr * KXS + xk] = xval ? x0 : 0.f;
  }
  float creg = cok ? c0v : 0.f;
  if (cok && a.cbuf) a.cbuf[(int64_t)cgr * H + cunit] = creg;
  if (tid < LR4 * KP) {
    const bool ok = hk < H && r0 + hr < B;
    const float v = ok ? h0v : 0.f;
    hS[0][he] = v;
    hS[1][he] = 0.f;
    if (ok) a.hbuf[(int64_t)(r0 + hr) * H + hk] = v;       // hbuf[0] = h0
  }
  int64_t xoff[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int gr = r0 + i < B ? r0 + i : B - 1;
    xoff[i] = (int64_t)gr * G4 + colc;
  }
  float xp[4] = {0.f, 0.f, 0.f, 0.f};
  if (KX == 0 && a.S > 0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) xp[i] = a.xproj[xoff[i]];
  }
  __syncthreads();
  LSTM_TICK(6);                                  // prologue (weights, x_0, c0 / h0)
  // x_t W_ih^T does not depend on h_{t-1}: its MFMAs for step t+1 are issued
  // right after step t's pre-activations are published, so the matrix pipe
  // works through them while the same waves run the cell update (VALU /
  // transcendentals / stores).  Same chains, same k order as issuing them at
  // the top of step t+1: bit-identical results.
  f32x4 acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto x_part = [&](int tt) {
    if constexpr (KX > 0) {
      // the same LDS read ring as the h part below: the wave issues these
      // MFMAs ahead of its cell update, so LDS round trips here delay the cell
      const float4* xr4 = reinterpret_cast<const float4*>(xS[tt & 1] + (lane & 3) * KXS);
      constexpr int NQX = KX / 4;
      float4 q[LSTM_HQ];
#pragma unroll
      for (int j = 0; j < LSTM_HQ && j < NQX; ++j) q[j] = xr4[j];
#pragma unroll
      for (int j = 0; j < NQX; ++j) {
        const float4 u = q[j % LSTM_HQ];
        const int ab = (j & 1) * 4;
        acc[ab + 0] = mfma4x64(u.x, wx[4 * j + 0], acc[ab + 0]);
        acc[ab + 1] = mfma4x64(u.y, wx[4 * j + 1], acc[ab + 1]);
        acc[ab + 2] = mfma4x64(u.z, wx[4 * j + 2], acc[ab + 2]);
        acc[ab + 3] = mfma4x64(u.w, wx[4 * j + 3], acc[ab + 3]);
        if (j + LSTM_HQ < NQX) q[j % LSTM_HQ] = xr4[j + LSTM_HQ];
      }
      __builtin_amdgcn_sched_group_barrier(0x100, LSTM_HQ < NQX ? LSTM_HQ : NQX, 0);
#pragma unroll
      for (int j = 0; j < NQX; ++j) {
        __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
        if (j + LSTM_HQ < NQX) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
    }
  };
  if (cact && a.S > 0) x_part(0);
  for (int t = 0; t < a.S; ++t) {
    const float* hp = hS[t & 1];
    float* hn = hS[(t + 1) & 1];
    if (cact) {
      const float4* hr = reinterpret_cast<const float4*>(hp + (lane & 3) * KP);
      // h_{t-1} through a ring of LSTM_HQ float4 LDS reads in flight (the
      // compiler's own schedule kept one read ahead, so every 4 MFMAs (32
      // cycles) waited out an LDS round trip); the same MFMAs per accumulator
      // in the same k order: float4 j feeds acc[4 (j & 1) .. + 3]
      constexpr int NQ = KP / 4;
      float4 q[LSTM_HQ];
#pragma unroll
      for (int j = 0; j < LSTM_HQ; ++j) q[j] = hr[j];
#pragma unroll
      for (int j = 0; j < NQ; ++j) {
        const float4 u = q[j % LSTM_HQ];
        const int ab = (j & 1) * 4;
        acc[ab + 0] = mfma4x64(u.x, w[4 * j + 0], acc[ab + 0]);
        acc[ab + 1] = mfma4x64(u.y, w[4 * j + 1], acc[ab + 1]);
        acc[ab + 2] = mfma4x64(u.z, w[4 * j + 2], acc[ab + 2]);
        acc[ab + 3] = mfma4x64(u.w, w[4 * j + 3], acc[ab + 3]);
        if (j + LSTM_HQ < NQ) q[j % LSTM_HQ] = hr[j + LSTM_HQ];
      }
      // pin that schedule (left alone, the scheduler shrinks the ring back to
      // one read for register pressure): the ring's first reads, then per
      // float4 its 4 MFMAs and the read that refills its slot
      __builtin_amdgcn_sched_group_barrier(0x100, LSTM_HQ, 0);
#pragma unroll
      for (int j = 0; j < NQ; ++j) {
        __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
        if (j + LSTM_HQ < NQ) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
      const f32x4 sum = ((acc[0] + acc[1]) + (acc[2] + acc[3])) +
                        ((acc[4] + acc[5]) + (acc[6] + acc[7]));
      if (col < G4) {
#pragma unroll
        for (int i = 0; i < 4; ++i) pre[i][col] = xp[i] + (sum[i] + bh);
      }
      if (KX == 0 && t + 1 < a.S) {
#pragma unroll
        for (int i = 0; i < 4; ++i) xp[i] = a.xproj[(int64_t)(t + 1) * B * G4 + xoff[i]];
      }
    }
    if constexpr (KX > 0) {   // x_{t+1} into the other buffer, x_{t+2} in flight
      if (xown && t + 1 < a.S) xS[(t + 1) & 1][xr * KXS + xk] = xval ? xnext : 0.f;
      if (xown && t + 2 < a.S) xnext = xload(t + 2);
    }
    LSTM_TICK(0);
    __syncthreads();
    if (cact) {               // next step's chains: x_{t+1} part now (see above)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (t + 1 < a.S) x_part(t + 1);
    }
    if (cell) {
      const float ig = sigm(pre[crow][cunit]), fg = sigm(pre[crow][H + cunit]);
      const float cg = ftanh(pre[crow][2 * H + cunit]), og = sigm(pre[crow][3 * H + cunit]);
      const float c = fg * creg + ig * cg;
      const float h = og * ftanh(c);
      creg = cok ? c : 0.f;
      hn[crow * KP + cunit] = cok ? h : 0.f;
      if (cok) {
        a.hbuf[(int64_t)(t + 1) * BH + (int64_t)cgr * H + cunit] = h;
        if (a.cbuf && t < keepS) a.cbuf[(int64_t)(t + 1) * BH + (int64_t)cgr * H + cunit] = c;
        if (a.gates && t < keepS) {
          float* gp = a.gates + ((int64_t)t * B + cgr) * G4 + cunit;
          gp[0] = ig; gp[H] = fg; gp[2 * H] = cg; gp[3 * H] = og;
        }
      }
    }
    LSTM_TICK(1);
    __syncthreads();
    LSTM_TICK(2);
  }
}

// KW: k range per wave (4H / waves-per-unit-group) rounded up to 8
template <int KW>
__global__ void __launch_bounds__(kWG8)
lstm_bwd_r4_kernel(LstmBwdArgs a) {
  if (a.skip && a.skip[0] != 0) return;
  LSTM_T0();
  constexpr int G4P = 4 * 128 + KW;               // dG row stride (reads run up to KW past 4H)
  __shared__ __attribute__((aligned(16))) float dG[LR4 * G4P];
  __shared__ float red[8][LR4][64];
  const int H = a.H, B = a.B, G4 = 4 * H;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r0 = blockIdx.x * LR4;
  const int64_t BH = (int64_t)B * H;
  const int NU = (H + 63) >> 6;                   // unit groups of 64 lanes
  const int WPG = 8 / NU;                         // waves per group (NU <= 2)
  const int kw = (G4 + WPG - 1) / WPG;
  const int ug = wave / WPG, kp = wave - ug * WPG;
  const int k0 = kp * kw;
  const int unit = ug * 64 + lane;
  const int uc = unit < H ? unit : H - 1;
  for (int e = tid; e < LR4 * G4P; e += kWG8) dG[e] = 0.f;
  float w[KW];                                    // W_hh[k0 + j][unit]
#pragma unroll
  for (int j = 0; j < KW; ++j) {
    const int k = k0 + j;
    const bool ok = j < kw && k < G4 && unit < H;
    const float x = a.w_hh[(int64_t)(k < G4 ? k : G4 - 1) * H + uc];
    w[j] = ok ? x : 0.f;
  }
  const bool cell = tid < LR4 * H;
  const int crow = cell ? tid / H : 0;
  const int cunit = cell ? tid - crow * H : 0;
  const int cgr = r0 + crow;
  const bool cok = cell && cgr < B;
  const int64_t grc = cgr < B ? cgr : B - 1;
  const int cug = cunit >> 6, cl = cunit & 63;
  float pg[4], pc = 0.f, pcp = 0.f, pdh = 0.f;
  auto fetch = [&](int t) {
    const float* gp = a.gates + ((int64_t)t * B + grc) * G4 + cunit;
    pg[0] = gp[0]; pg[1] = gp[H]; pg[2] = gp[2 * H]; pg[3] = gp[3 * H];
    pc = a.cbuf[(int64_t)(t + 1) * BH + grc * H + cunit];
    pcp = a.cbuf[(int64_t)t * BH + grc * H + cunit];
    pdh = a.dh[(int64_t)t * BH + grc * H + cunit];
  };
  if (cell && a.S > 0) fetch(a.S - 1);
  float dcreg = 0.f;
  __syncthreads();
  LSTM_TICK(7);                                  // prologue (W_hh, first step inputs)
  for (int t = a.S - 1; t >= 0; --t) {
    if (cell) {
      float dhr = 0.f;
      if (t < a.S - 1) {
        for (int p = 0; p < WPG; ++p) dhr += red[cug * WPG + p][crow][cl];
      }
      const float ig = pg[0], fg = pg[1], cg = pg[2], og = pg[3];
      const float dh = pdh + dhr;
      const float tc = ftanh(pc);
      const float dc = dh * og * (1.f - tc * tc) + dcreg;
      const float d_o = (dh * tc) * (og * (1.f - og));
      const float d_i = (dc * cg) * (ig * (1.f - ig));
      const float d_g = (dc * ig) * (1.f - cg * cg);
      const float d_f = (dc * pcp) * (fg * (1.f - fg));
      dcreg = cok ? dc * fg : 0.f;
      float* l = dG + crow * G4P + cunit;
      l[0] = cok ? d_i : 0.f; l[H] = cok ? d_f : 0.f;
      l[2 * H] = cok ? d_g : 0.f; l[3 * H] = cok ? d_o : 0.f;
      if (cok) {
        float* o = a.dgates + ((int64_t)t * B + cgr) * G4 + cunit;
        o[0] = d_i; o[H] = d_f; o[2 * H] = d_g; o[3 * H] = d_o;
      }
      if (t > 0) fetch(t - 1);
    }
    LSTM_TICK(3);
    __syncthreads();
    LSTM_TICK(4);
    if (t == 0) break;
    if (wave < NU * WPG) {
      f32x4 acc[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
      // dgates operand reads LQ float4 ahead (as in the forward's h loop)
      constexpr int NQ = KW / 4, LQ = 4;
      const float4* dr = reinterpret_cast<const float4*>(dG + (lane & 3) * G4P + k0);
      float4 q[LQ];
#pragma unroll
      for (int j = 0; j < LQ && j < NQ; ++j) q[j] = dr[j];
#pragma unroll
      for (int j = 0; j < NQ; ++j) {
        const float4 u = q[j % LQ];
        if (j + LQ < NQ) q[j % LQ] = dr[j + LQ];
        const int a0 = (j & 1) * 4;
        acc[a0 + 0] = mfma4x64(u.x, w[4 * j + 0], acc[a0 + 0]);
        acc[a0 + 1] = mfma4x64(u.y, w[4 * j + 1], acc[a0 + 1]);
        acc[a0 + 2] = mfma4x64(u.z, w[4 * j + 2], acc[a0 + 2]);
        acc[a0 + 3] = mfma4x64(u.w, w[4 * j + 3], acc[a0 + 3]);
        __builtin_amdgcn_sched_barrier(0);
      }
      const f32x4 sum = ((acc[0] + acc[1]) + (acc[2] + acc[3])) +
                        ((acc[4] + acc[5]) + (acc[6] + acc[7]));
#pragma unroll
      for (int i = 0; i < 4; ++i) red[wave][i][lane] = sum[i];
    }
    LSTM_TICK(5);
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// VALU variants for small local batches (strong scaling: a rank of the N = 8
// C3 job holds 128 segments).  The MFMA forms above waste the recurrence's
// matrix pipe at few segments per workgroup (v_mfma_f32_4x4x1 always computes
// 4 rows) and a step's latency does not fall with the batch.  Here a
// workgroup owns R <= 4 segments and thread (u, q) = 4u + q owns ONE gate
// column g = q*H + u (gate q of hidden unit u) with its W_hh row (and, fused,
// its W_ih row) in registers:
//   pre_g   = x_t W_ih[g] + b_ih[g] + h_{t-1} W_hh[g] + b_hh[g]   (FMA chains,
//             h_{t-1} broadcast from LDS as 16-byte reads)
//   a_g     = sigmoid / tanh (gate g lives in lane 4u + q)
//   i,f,g,o of unit u gathered inside the lane quad with DPP quad broadcasts
//   c, h    computed redundantly by the quad's 4 lanes (identical values)
// so a step is one matvec, one quad exchange and ONE barrier (h_t published
// to LDS).  With R = 1 the 128-segment batch fills 128 CUs and a step is ~100
// dependent-free FMAs per thread.  The x part of step t+1 (independent of
// h_t) is formed after h_t is published, in the barrier's shadow.
// Backward: thread (u, q) holds column u of W_hh restricted to gate q's rows,
// dh_rec[u] = sum_q sum_j dgates[q*H + j] W_hh[q*H + j][u] is a per-lane
// partial over gate q plus a fixed-order quad sum.
#endif  // SMI_LSTM_MFMA

#if SMI_LSTM_VALU_HALF

// s0..s3 += v[k] * w[k] over k < KP, v read from LDS as KP / 4 float4s in
// chunks of kVC, the next chunk's reads issued before the current chunk's FMAs
#ifndef SMI_LSTM_VC
#define SMI_LSTM_VC 4
#endif
constexpr int kVC = SMI_LSTM_VC;
// SMI_LSTM_PK=1: the dot products on v_pk_fma_f32 (same sums, half the
// instructions) — measured slower at 128 segments (1.70 / 1.61 us per forward /
// BPTT step against 1.62 / 1.50 on scalar FMAs): A/B only
#ifndef SMI_LSTM_PK
#define SMI_LSTM_PK 0
#endif
template <int KP>
__device__ __forceinline__ void v_dot_pipelined(const float4* __restrict__ v, const float (&w)[KP],
                                                float& s0, float& s1, float& s2, float& s3) {
  constexpr int N4 = KP / 4, NC = (N4 + kVC - 1) / kVC;
  float4 buf[2][kVC];
#if SMI_LSTM_PK
  vf2 a01 = {s0, s1}, a23 = {s2, s3};
#endif
  auto ld = [&](int c) {
#pragma unroll
    for (int i = 0; i < kVC; ++i)
      if (c * kVC + i < N4) buf[c & 1][i] = v[c * kVC + i];
  };
  ld(0);
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    if (c + 1 < NC) ld(c + 1);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < kVC; ++i) {
      const int k4 = c * kVC + i;
      if (k4 < N4) {
        const float4 hv = buf[c & 1][i];
#if SMI_LSTM_PK
        // v_pk_fma_f32: (s0, s1) and (s2, s3) as packed pairs, each lane an
        // fmaf of the same operands as the scalar form (bit-identical sums)
        a01 = __builtin_elementwise_fma(vf2{hv.x, hv.y}, vf2{w[4 * k4], w[4 * k4 + 1]}, a01);
        a23 = __builtin_elementwise_fma(vf2{hv.z, hv.w}, vf2{w[4 * k4 + 2], w[4 * k4 + 3]}, a23);
#else
        s0 = fmaf(hv.x, w[4 * k4], s0);
        s1 = fmaf(hv.y, w[4 * k4 + 1], s1);
        s2 = fmaf(hv.z, w[4 * k4 + 2], s2);
        s3 = fmaf(hv.w, w[4 * k4 + 3], s3);
#endif
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  }
#if SMI_LSTM_PK
  s0 = a01.x; s1 = a01.y; s2 = a23.x; s3 = a23.y;
#endif
}

template <int R, int KP, int KX>
__global__ void __launch_bounds__(kVT)
lstm_fwd_v_kernel(LstmFwdArgs a) {
  if (a.skip && a.skip[0] != 0) return;
  const int keepS = a.keep > 0 ? a.keep : a.S;     // steps whose c / gates are stored
  constexpr int KXS = KX > 0 ? KX : 4;
  __shared__ __attribute__((aligned(16))) float hS[2][R * KP];
  // KX > 0: the segment rows' x for EVERY step, staged once before the
  // recurrence (S x R x KXS floats, dynamic LDS): the step loop then issues no
  // loads at all, so nothing in it waits on memory (a per-step prefetch made
  // each step wait for its own stores: vmcnt counts loads and stores in order).
  // Then every step's x part x_t W_ih[g] + biases is formed up front, off the
  // recurrence's critical path, into xP [S][R][blockDim] (each thread reads
  // back only its own values: no barrier).
  extern __shared__ __attribute__((aligned(16))) float xS[];
  float* xP = xS + (((int64_t)a.S * R * KXS + 3) & ~3);
  const int H = a.H, B = a.B, G4 = 4 * H;
  const int tid = threadIdx.x, u = tid >> 2, q = tid & 3;
  const bool act = u < H;
  const int uc = act ? u : H - 1;
  const int g = q * H + uc;
  const int r0 = blockIdx.x * R;
  const int64_t BH = (int64_t)B * H;
  float w[KP];
#pragma unroll
  for (int k = 0; k < KP; ++k) {
    const float x = a.w_hh[(int64_t)g * H + (k < H ? k : H - 1)];
    w[k] = k < H ? x : 0.f;
  }
  float bh = a.b_hh[g];
  float wx[KXS];
  if constexpr (KX > 0) {
#pragma unroll
    for (int k = 0; k < KX; ++k) {
      const float x = a.w_ih[(int64_t)g * a.din + (k < a.din ? k : a.din - 1)];
      wx[k] = k < a.din ? x : 0.f;
    }
    bh += a.b_ih[g];
  }
  int bseg[R];
  bool okr[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    okr[r] = act && r0 + r < B;
    bseg[r] = r0 + r < B ? r0 + r : B - 1;
  }
  // x staging (KX > 0): thread e < R*KX owns (row e / KX, k e % KX) of x_t
  if constexpr (KX > 0) {
    for (int e = tid; e < a.S * R * KXS; e += blockDim.x) {
      const int t = e / (R * KXS), q = e - t * (R * KXS);
      const int r = q / KXS, k = q - r * KXS;
      float v = 0.f;
      if (k < a.din && r0 + r < B) v = a.x[((int64_t)t * B + r0 + r) * a.ldx + k];
      xS[e] = v;
    }
  }
  float creg[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    creg[r] = a.c0[(int64_t)bseg[r] * H + uc];
    if (okr[r] && q == 0 && a.cbuf) a.cbuf[(int64_t)bseg[r] * H + u] = creg[r];
  }
  for (int e = tid; e < R * KP; e += blockDim.x) {
    const int r = e / KP, k = e - r * KP;
    const bool ok = k < H && r0 + r < B;
    const float v = ok ? a.h0[(int64_t)(r0 + r) * H + k] : 0.f;
    hS[0][e] = v;
    hS[1][e] = 0.f;
    if (ok) a.hbuf[(int64_t)(r0 + r) * H + k] = v;          // hbuf[0] = h0
  }
  __syncthreads();
  // x part of step t (+ the combined bias)
  float xacc[R];
  auto x_part = [&](int t) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if constexpr (KX > 0) {
        const float4* xp = reinterpret_cast<const float4*>(xS + (t * R + r) * KXS);
        float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
#pragma unroll
        for (int k4 = 0; k4 < KX / 4; ++k4) {
          const float4 v = xp[k4];
          s0 = fmaf(v.x, wx[4 * k4], s0);
          s1 = fmaf(v.y, wx[4 * k4 + 1], s1);
          s2 = fmaf(v.z, wx[4 * k4 + 2], s2);
          s3 = fmaf(v.w, wx[4 * k4 + 3], s3);
          if ((k4 & 3) == 3) __builtin_amdgcn_sched_barrier(0);
        }
        xacc[r] = (s0 + s1) + (s2 + s3);
      } else {
        xacc[r] = a.xproj[((int64_t)t * B + bseg[r]) * G4 + g];
      }
    }
  };
  float xpn[R];                                  // KX == 0: xproj of step t+1, in flight
  if constexpr (KX > 0) {
    for (int t = 0; t < a.S; ++t) {
      x_part(t);
#pragma unroll
      for (int r = 0; r < R; ++r) xP[(t * R + r) * blockDim.x + tid] = xacc[r];
    }
  } else {
    if (a.S > 0) x_part(0);
  }
  // drain the prologue's loads here: otherwise the waitcnt pass sees the c0
  // load (creg) possibly in flight at the loop header and puts a vmcnt(0)
  // INSIDE the loop, before every step's cell update
  __builtin_amdgcn_s_waitcnt(0x0F70);            // vmcnt(0)
  for (int t = 0; t < a.S; ++t) {
    const float* hp = hS[t & 1];
    float* hn = hS[(t + 1) & 1];
    // x_{t+2}: issued before this step's stores, so the LDS write at the end
    // of the step waits for this load only (vmcnt counts in issue order)
    if constexpr (KX == 0) {       // xproj of step t+1, issued before this step's stores
#pragma unroll
      for (int r = 0; r < R; ++r)
        xpn[r] = a.xproj[((int64_t)(t + 1 < a.S ? t + 1 : t) * B + bseg[r]) * G4 + g];
    } else {
#pragma unroll
      for (int r = 0; r < R; ++r) xacc[r] = xP[(t * R + r) * blockDim.x + tid];
    }
    // one segment after the other (a sched_barrier between them): interleaving
    // the R matvecs keeps R x (h reads + accumulators) live next to the
    // KP + KX weight registers and spills from R = 2
#pragma unroll
    for (int r = 0; r < R; ++r) {
      float acc0 = 0.f, acc1 = 0.f, acc2 = 0.f, acc3 = 0.f;
      // h_{t-1} in chunks of kVC 16-byte LDS reads, software-pipelined one
      // chunk ahead into two register sets: the FMAs of chunk c run while the
      // reads of chunk c + 1 are in flight (lgkmcnt(kVC) instead of a full
      // drain per chunk); the sched_barriers keep the compiler from hoisting
      // every read of the step (which needs KP more VGPRs than the weights leave)
      const float4* hp4 = reinterpret_cast<const float4*>(hp + r * KP);
      v_dot_pipelined<KP>(hp4, w, acc0, acc1, acc2, acc3);
      const float pre = xacc[r] + (((acc0 + acc1) + (acc2 + acc3)) + bh);
      const float av = q == 2 ? ftanh(pre) : sigm(pre);
      const float ig = quad_bcast<0>(av), fg = quad_bcast<1>(av);
      const float cg = quad_bcast<2>(av), og = quad_bcast<3>(av);
      const float c = fg * creg[r] + ig * cg;
      const float h = og * ftanh(c);
      creg[r] = c;
      if (okr[r]) {
        const int b = bseg[r];
        if (q == 0) {
          hn[r * KP + u] = h;
          a.hbuf[(int64_t)(t + 1) * BH + (int64_t)b * H + u] = h;
          if (a.cbuf && t < keepS) a.cbuf[(int64_t)(t + 1) * BH + (int64_t)b * H + u] = c;
        }
        if (a.gates && t < keepS) a.gates[((int64_t)t * B + b) * G4 + g] = av;
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (KX == 0) {
#pragma unroll
      for (int r = 0; r < R; ++r) xacc[r] = xpn[r];
    }
    __syncthreads();
  }
}

template <int R, int KP>
__global__ void __launch_bounds__(kVT)
lstm_bwd_v_kernel(LstmBwdArgs a) {
  if (a.skip && a.skip[0] != 0) return;
  __shared__ __attribute__((aligned(16))) float dG[2][R * 4 * KP];
  const int H = a.H, B = a.B, G4 = 4 * H;
  const int tid = threadIdx.x, u = tid >> 2, q = tid & 3;
  const bool act = u < H;
  const int uc = act ? u : H - 1;
  const int g = q * H + uc;
  const int r0 = blockIdx.x * R;
  const int64_t BH = (int64_t)B * H;
  for (int e = tid; e < 2 * R * 4 * KP; e += blockDim.x) (&dG[0][0])[e] = 0.f;
  float w[KP];                                   // W_hh[q*H + j][u]
#pragma unroll
  for (int j = 0; j < KP; ++j) {
    const float x = a.w_hh[(int64_t)(q * H + (j < H ? j : H - 1)) * H + uc];
    w[j] = j < H ? x : 0.f;
  }
  int bseg[R];
  bool okr[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    okr[r] = act && r0 + r < B;
    bseg[r] = r0 + r < B ? r0 + r : B - 1;
  }
  // per-step inputs, fetched two steps ahead into alternating register sets:
  // a step's loads are issued right after its dgates store and used two steps
  // later, so neither their latency nor the stores ahead of them (vmcnt counts
  // loads and stores in issue order) reach the critical path
  struct In { float gq[R], ct[R], ctm[R], dho[R]; };
  In A, Bn;
  float dcreg[R], dhr[R];
  auto fetch = [&](int t, In& X) {               // t clamped by the caller: always issued
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int64_t b = bseg[r];
      X.gq[r] = a.gates[((int64_t)t * B + b) * G4 + g];
      X.ct[r] = a.cbuf[(int64_t)(t + 1) * BH + b * H + uc];
      X.ctm[r] = a.cbuf[(int64_t)t * BH + b * H + uc];
      X.dho[r] = a.dh[(int64_t)t * BH + b * H + uc];
    }
  };
#pragma unroll
  for (int r = 0; r < R; ++r) dcreg[r] = dhr[r] = 0.f;
  if (a.S <= 0) return;
  fetch(a.S - 1, A);
  fetch(a.S >= 2 ? a.S - 2 : 0, Bn);
  __syncthreads();
  // one step; false after step 0
  auto step = [&](int t, In& X) -> bool {
    float* dgw = dG[t & 1];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const float ig = quad_bcast<0>(X.gq[r]), fg = quad_bcast<1>(X.gq[r]);
      const float cg = quad_bcast<2>(X.gq[r]), og = quad_bcast<3>(X.gq[r]);
      const float dh = X.dho[r] + dhr[r];
      const float tc = ftanh(X.ct[r]);
      const float dc = dh * og * (1.f - tc * tc) + dcreg[r];
      const float d_o = (dh * tc) * (og * (1.f - og));
      const float d_i = (dc * cg) * (ig * (1.f - ig));
      const float d_g = (dc * ig) * (1.f - cg * cg);
      const float d_f = (dc * X.ctm[r]) * (fg * (1.f - fg));
      dcreg[r] = okr[r] ? dc * fg : 0.f;
      float dq = q == 0 ? d_i : q == 1 ? d_f : q == 2 ? d_g : d_o;
      dq = okr[r] ? dq : 0.f;
      if (act) dgw[r * 4 * KP + q * KP + u] = dq;
      if (okr[r]) a.dgates[((int64_t)t * B + bseg[r]) * G4 + g] = dq;
    }
    fetch(t >= 2 ? t - 2 : 0, X);
    __syncthreads();
    if (t == 0) return false;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const float4* dp = reinterpret_cast<const float4*>(dgw + r * 4 * KP + q * KP);
      float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
      v_dot_pipelined<KP>(dp, w, s0, s1, s2, s3);
      const float p = (s0 + s1) + (s2 + s3);
      // fixed-order quad sum: every lane of the quad gets the same dh_rec
      dhr[r] = (quad_bcast<0>(p) + quad_bcast<1>(p)) + (quad_bcast<2>(p) + quad_bcast<3>(p));
    }
    return true;
  };
  for (int t = a.S - 1; t >= 0; t -= 2) {
    if (!step(t, A)) break;
    if (!step(t - 1, Bn)) break;
  }
}


// ---------------------------------------------------------------------------
// One segment per workgroup with the recurrent product's K split over the
// lane quad (round 5; R = 1 — a rank's share of a strong-scaled job).  The
// R-segment kernels above give thread (u, q) a whole W_hh row, so every
// thread reads all of h_{t-1} each step (26 ds_read_b128 per wave at H = 100:
// 728 LDS cycles per CU per step) and runs one 104-long FMA stream.  Here
// thread (u, q) = (tid >> 2, tid & 3) holds the FOUR gate rows j*H + u of
// unit u over its quarter k in [q*KQ, (q+1)*KQ) as (k, k+1) pairs:
//   forward  p_j = sum_k h_{t-1}[k] W_hh[j*H + u][k] on v_pk_fma_f32 (KQ/2
//            packed FMAs per gate over 2-float LDS reads: 13 ds_read_b64 per
//            wave), the four lanes' partials summed by two quad DPP adds
//            (l ^ 1, then l ^ 2: every lane of the quad ends with the same
//            four sums); lane q then finishes gate q exactly as the R forms
//            do (activation, quad broadcast, the cell computed alike in the
//            four lanes).  The x part is precomputed with the same K split of
//            W_ih over the staged x sequence (XQ > 0), or read from xproj
//            (XQ == 0) one step ahead.  W_hh is loaded while the x parts are
//            formed; the step's hbuf / cbuf / gates stores are issued after
//            the barrier, behind the next step's LDS reads.
//   BPTT     thread (ug, rr) = (tid >> 4, tid & 15) holds W_hh[r][4ug..4ug+3]
//            for the rows r in [rr*BR, rr*BR + BR) (BR = ceil(H / 4)), reads
//            those BR dgates of the step (a [16][BRP] padded LDS image: b128
//            reads, 64 distinct banks) and sums its four units on packed
//            FMAs; the 16 partials of a unit meet through four DPP adds
//            (quad l ^ 1, l ^ 2, row half-mirror, row rotate 8: identical
//            sums in all 16 lanes), and the cell backward keeps the (u, q)
//            mapping (unit u's sum sits in its own 16-lane row).
// Measured (tools/exp/lstm_v_exp.hip, 128 segments, H 100, one MI355X): see
// DESIGN.md §9.  Sums are fixed-order (deterministic); their association
// differs from the R forms' (fp32 rounding only).
// a1: a second, independent sequence set in the same launch (workgroups >=
// a0.B: the GAE critic pass and the reference policy's forward, two weight
// sets over two inputs); single launches pass a0 twice over a0.B workgroups
// A4 (x staged, XQ > 0): every lane finishes all four gates of its unit (after
// the two quad DPP adds each lane holds all four sums, and xP keeps unit u's
// four x parts at 4u .. 4u + 3): four independent activations instead of one
// followed by four quad broadcasts on the step's dependent chain (same ops on
// the same values: bit-identical)
template <int KQ, int XQ, bool XM, int WI, bool A4 = false>
__global__ void __launch_bounds__(kVT)
lstm_fwd_q_kernel(LstmFwdArgs a0, LstmFwdArgs a1) {
  static_assert(!A4 || XQ > 0, "A4 reads the staged x parts");
  static_assert(WI != 2 || KQ % 4 == 0, "float4 k runs");
  const bool second = (int)blockIdx.x >= a0.B;
  const LstmFwdArgs& a = second ? a1 : a0;
  const int b = second ? (int)blockIdx.x - a0.B : (int)blockIdx.x;
  // the skip flag is read with the prologue's loads and tested before the
  // first global store (its own round trip in front of them cost ~1 us)
  const int skipv = a.skip ? a.skip[0] : 0;
  LSTM_T0();
  const int keepS = a.keep > 0 ? a.keep : a.S;
  static_assert(KQ % 2 == 0 && XQ % 4 == 0, "K split: pairs of h, float4 runs of x");
  constexpr int KX = 4 * XQ, KXS = XQ > 0 ? KX : 4;
  __shared__ __attribute__((aligned(16))) float hS[2][4 * KQ];
  extern __shared__ __attribute__((aligned(16))) float xS[];    // [S][KXS] x, then [S][blockDim] x parts
  float* xP = xS + (((int64_t)a.S * KXS + 3) & ~3);
  const int H = a.H, B = a.B, G4 = 4 * H, NT = blockDim.x;
  const int tid = threadIdx.x, u = tid >> 2, q = tid & 3;
  const bool act = u < H;
  const int uc = act ? u : H - 1;
  const int g = q * H + uc;
  const int64_t BH = (int64_t)B * H;
  // Round 6: the prologue issues all of its loads (biases, c0 / h0, the
  // matrix-core W_ih operands, the x sequence) before waiting on any, each
  // unconditionally from a clamped address with nothing selected on it
  // afterwards.  A load whose value was used under a per-lane condition was
  // sunk into its own exec-masked branch with a vmcnt(0) wait at the merge,
  // and loads behind a dependent store waited for it: one memory round trip
  // per load group.  Padding needs no select: a weight loaded for k past the
  // row (or for a gate row / unit past the shape) only ever multiplies a zero
  // of the LDS-staged x / h images (or feeds a result that is dropped), and
  // x * 0 = +-0 leaves every sum bit-identical; the staged x / h0 images get
  // their zeros by a multiply.
  // the x sequence's first XB * NT elements (all of it up to S * KX = 7168
  // at KX 48 on 448 threads), issued first; stored to LDS after the rest
  constexpr int XB = 4;                           // x loads in flight per thread
  float xv[XB];
  if constexpr (XQ > 0) {
#pragma unroll
    for (int j = 0; j < XB; ++j) {
      const int e = min(tid + j * NT, a.S * KX - 1);
      const int t = e / KX, k = e - t * KX;
      xv[j] = a.x[((int64_t)t * B + b) * a.ldx + min(k, a.din - 1)];
    }
  }
  const float bhh = a.b_hh[g];
  const float bih = XQ > 0 ? a.b_ih[g] : 0.f;
  const float creg0 = a.c0[(int64_t)b * H + uc];
  const float h0v = a.h0[(int64_t)b * H + min(tid, H - 1)];   // (NT >= 4 KQ: one h0 slot per thread)
  // the matrix-core x parts' B operands (W_ih^T, below) and bias sums, issued
  // before W_hh's so that the x parts wait on them alone: wave w's gate tiles
  // w + ti*NW (ti < 4 covers ceil(H/4) tiles over ceil(H/16) waves).  The k
  // order is permuted so a lane's operands are contiguous: MFMA step s of lane
  // l takes k = 16 (s >> 2) + 4 (l >> 4) + (s & 3) (A from the staged x rows
  // alike), so the four lane groups of a row read 64 contiguous bytes per k
  // chunk
  constexpr int XT = 4, KS = KX / 4;
  constexpr bool XMF = XQ > 0 && XM;
  float bw[XMF ? XT : 1][XMF ? KS : 1];
  float bbi[XMF ? XT : 1], bbh[XMF ? XT : 1];
  if constexpr (XMF) {
    const int lane = tid & 63, wave = tid >> 6, NW = NT >> 6;
    // float2 runs (the dispatcher takes this form only for an even din and an
    // 8-byte aligned W_ih); k >= din and gate rows >= G4 load clamped (finite)
    // weights: they meet the zero x columns / are dropped with their output rows
#pragma unroll
    for (int ti = 0; ti < XT; ++ti) {
      const int gg = min((wave + ti * NW) * 16 + (lane & 15), G4 - 1);
      const float* wr = a.w_ih + (int64_t)gg * a.din;
#pragma unroll
      for (int m = 0; m < KS / 4; ++m) {
        const int k0 = 16 * m + 4 * (lane >> 4);
        const float2 p0 = *reinterpret_cast<const float2*>(wr + min(k0, a.din - 2));
        const float2 p1 = *reinterpret_cast<const float2*>(wr + min(k0 + 2, a.din - 2));
        bw[ti][4 * m] = p0.x; bw[ti][4 * m + 1] = p0.y;
        bw[ti][4 * m + 2] = p1.x; bw[ti][4 * m + 3] = p1.y;
      }
      bbi[ti] = a.b_ih[gg];
      bbh[ti] = a.b_hh[gg];
    }
  }
  // W_hh rows j*H + u over the k pairs (8i + 2q, 8i + 2q + 1), i < KQ / 2: the
  // quad's four lanes read 32 contiguous bytes of a row per load (a lane-
  // contiguous quarter row put every lane of a load on its own cache line: the
  // prologue re-fetched W_hh from L2 many times over); issued last of the
  // prologue's loads, in flight through the x staging and the x parts
  vf2 wv[4][KQ / 2];
  // The vector width is the dispatcher's (fwd_q_dispatch: WI 2 needs H % 4 ==
  // 0 and a 16-byte aligned W_hh, WI 1 H even and 8 bytes).  A run-time
  // vec / scalar branch here was merged by the compiler into one path of
  // single-dword loads with selected addresses: 112 load instructions per lane
  // instead of 28, each touching 16 rows (13 us of the prologue, round 6).
  if constexpr (WI == 2) {
    // k runs (16 i + 4q .. + 3): 64 contiguous bytes of a row per quad and load;
    // k past H: a clamped (finite) weight times the zero h padding
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float* r = a.w_hh + (int64_t)(j * H + uc) * H;
#pragma unroll
      for (int i = 0; i < KQ / 4; ++i) {
        const float4 v = *reinterpret_cast<const float4*>(r + min(16 * i + 4 * q, H - 4));
        wv[j][2 * i] = vf2{v.x, v.y};
        wv[j][2 * i + 1] = vf2{v.z, v.w};
      }
    }
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float* r = a.w_hh + (int64_t)(j * H + uc) * H;
#pragma unroll
      for (int i = 0; i < KQ / 2; ++i) {
        const int k = WI ? 8 * i + 2 * q : q * KQ + 2 * i;
        if constexpr (WI == 1) {
          const float2 t2 = *reinterpret_cast<const float2*>(r + min(k, H - 2));
          wv[j][i] = vf2{t2.x, t2.y};
        } else {
          wv[j][i] = vf2{r[min(k, H - 1)], r[min(k + 1, H - 1)]};
        }
      }
    }
  }
  if constexpr (XQ > 0) {
    // stored unconditionally at the clamped index (a thread past the end
    // writes the owner's own value; a store under a per-lane condition let the
    // compiler sink its load into the branch, with a vmcnt(0) at the merge)
#pragma unroll
    for (int j = 0; j < XB; ++j) {
      const int e = min(tid + j * NT, a.S * KX - 1);
      xS[e] = xv[j] * (float)(e % KX < a.din);
    }
    for (int e0 = tid + XB * NT; e0 < a.S * KX; e0 += XB * NT) {     // longer sequences
      float v[XB];
#pragma unroll
      for (int j = 0; j < XB; ++j) {
        const int e = min(e0 + j * NT, a.S * KX - 1);
        const int t = e / KX, k = e - t * KX;
        v[j] = a.x[((int64_t)t * B + b) * a.ldx + min(k, a.din - 1)];
      }
#pragma unroll
      for (int j = 0; j < XB; ++j) {
        const int e = e0 + j * NT;
        if (e < a.S * KX) xS[e] = v[j] * (float)(e % KX < a.din);
      }
    }
  }
  if (skipv != 0) return;                        // (uniform)
  const float bh = bhh + bih;
  float creg = creg0;
  if (act && q == 0 && a.cbuf) a.cbuf[(int64_t)b * H + u] = creg;
  {
    // (clamped like the x stores: 4 KQ >= H, so a thread past 4 KQ writes the
    // value slot 4 KQ - 1 holds)
    const int e = min(tid, 4 * KQ - 1);
    hS[0][e] = h0v * (float)(e < H);
    hS[1][e] = 0.f;
    if (tid < H) a.hbuf[(int64_t)b * H + tid] = h0v;
  }
  __syncthreads();
  LSTM_TICK(0);                                  // x staged, c0 / h0, W_ih issued
  if constexpr (XMF) {
    // x parts of every step on the matrix cores: xP[t][tid(g)] = sum_k x_t[k]
    // W_ih[g][k] + b_ih[g] + b_hh[g] as v_mfma_f32_16x16x4_f32 tiles of 16 steps
    // x 16 gate rows (A = the staged x rows, B = W_ih^T, one k-ordered fmaf
    // chain per element); a tile's B operand stays in registers across the
    // step tiles
    const int lane = tid & 63, wave = tid >> 6, NW = NT >> 6;
    const int nmt = (a.S + 15) >> 4;
#pragma unroll
    for (int ti = 0; ti < XT; ++ti) {
      const int nt = wave + ti * NW;
      if (nt * 16 >= G4) break;
      const int gs = nt * 16 + (lane & 15);                 // the D column's gate
      const float bsum = bbi[ti] + bbh[ti];                  // (gs >= G4 dropped)
      const int dst = gs < G4 ? 4 * (gs % H) + gs / H : 0;
      auto x_tile = [&](int mt) {
        const int r = min(mt * 16 + (lane & 15), a.S - 1);
        const float4* xr = reinterpret_cast<const float4*>(xS + r * KX + 4 * (lane >> 4));
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
        // every k chunk (no early exit at din: columns past din are the zero
        // padding of the staged x, exact zeros in the sums), so a tile's LDS
        // reads issue together instead of one wait per chunk
#pragma unroll
        for (int m = 0; m < KS / 4; ++m) {
          const float4 xv = xr[4 * m];
          acc = __builtin_amdgcn_mfma_f32_16x16x4f32(xv.x, bw[ti][4 * m], acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_16x16x4f32(xv.y, bw[ti][4 * m + 1], acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_16x16x4f32(xv.z, bw[ti][4 * m + 2], acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_16x16x4f32(xv.w, bw[ti][4 * m + 3], acc, 0, 0, 0);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int t = mt * 16 + 4 * (lane >> 4) + i;
          if (t < a.S && gs < G4) xP[(int64_t)t * NT + dst] = acc[i] + bsum;
        }
      };
      // the step tiles unrolled (S <= 61 in this form: kVxMax), no loop back
      // edge for the waitcnt pass to merge over (the first tile had waited
      // vmcnt(0), i.e. on W_hh's loads as well as its own W_ih operands)
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
        if (mt < nmt) x_tile(mt);
      for (int mt = 4; mt < nmt; ++mt) x_tile(mt);
    }
    __syncthreads();
    LSTM_TICK(1);                                // x parts on the matrix cores
  } else if constexpr (XQ > 0) {
    // x parts of every step: W_ih rows j*H + u over x columns [q*XQ, q*XQ + XQ)
    float wx[4][XQ];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float* r = a.w_ih + (int64_t)(j * H + uc) * a.din;
#pragma unroll
      for (int kk = 0; kk < XQ; ++kk) {
        const int k = q * XQ + kk;
        wx[j][kk] = k < a.din ? r[k] : 0.f;
      }
    }
    for (int t = 0; t < a.S; ++t) {
      const float4* xp = reinterpret_cast<const float4*>(xS + t * KX + q * XQ);
      float pj[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int k4 = 0; k4 < XQ / 4; ++k4) {
        const float4 v = xp[k4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          pj[j] = fmaf(v.x, wx[j][4 * k4], pj[j]);
          pj[j] = fmaf(v.y, wx[j][4 * k4 + 1], pj[j]);
          pj[j] = fmaf(v.z, wx[j][4 * k4 + 2], pj[j]);
          pj[j] = fmaf(v.w, wx[j][4 * k4 + 3], pj[j]);
        }
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        pj[j] += dpp_x1(pj[j]);
        pj[j] += dpp_x2(pj[j]);
      }
      const float mine = q == 0 ? pj[0] : q == 1 ? pj[1] : q == 2 ? pj[2] : pj[3];
      xP[(int64_t)t * NT + tid] = mine + bh;
    }
  }
  __builtin_amdgcn_s_waitcnt(0x0F70);            // vmcnt(0): W_hh (and xproj of step 0) landed
  LSTM_TICK(2);                                  // W_hh wait
  float* hb = a.hbuf + BH + (int64_t)b * H + uc;
  float* cb = a.cbuf ? a.cbuf + BH + (int64_t)b * H + uc : nullptr;
  float* gp = a.gates ? a.gates + (int64_t)b * G4 + g : nullptr;
  const int64_t gstep = (int64_t)B * G4;
  float xnext = 0.f;
  if constexpr (XQ == 0) {
    if (a.S > 0) xnext = a.xproj[(int64_t)b * G4 + g];
  }
  float ph = 0.f, pc = 0.f, pav = 0.f;
  for (int t = 0; t < a.S; ++t) {
    const float* hp = hS[t & 1] + (WI == 2 ? 4 * q : WI ? 2 * q : q * KQ);
    float* hn = hS[(t + 1) & 1];
    float xacc = 0.f;
    float4 x4 = float4{0.f, 0.f, 0.f, 0.f};
    if constexpr (A4) {
      x4 = *reinterpret_cast<const float4*>(xP + (int64_t)t * NT + 4 * uc);
    } else if constexpr (XQ > 0) {
      xacc = xP[(int64_t)t * NT + tid];
    } else {
      xacc = xnext + bh;
    }
    float2 hv[KQ / 2];
    if constexpr (WI == 2) {
      const float4* h4 = reinterpret_cast<const float4*>(hp);
#pragma unroll
      for (int i = 0; i < KQ / 4; ++i) {
        const float4 v = h4[4 * i];
        hv[2 * i] = float2{v.x, v.y};
        hv[2 * i + 1] = float2{v.z, v.w};
      }
    } else {
      const float2* h2 = reinterpret_cast<const float2*>(hp);
#pragma unroll
      for (int i = 0; i < KQ / 2; ++i) hv[i] = h2[WI ? 4 * i : i];
    }
    if constexpr (XQ == 0) {          // xproj of step t + 1, in flight through the step
      if (t + 1 < a.S) xnext = a.xproj[((int64_t)(t + 1) * B + b) * G4 + g];
    }
    // the previous step's stores, behind this step's LDS reads
    if (t > 0 && act) {
      if (q == 0) {
        hb[0] = ph;
        hb += BH;
        if (cb && t - 1 < keepS) cb[0] = pc;
        if (cb) cb += BH;
      }
      if (gp && t - 1 < keepS) gp[0] = pav;
      if (gp) gp += gstep;
    }
    vf2 pp[4] = {vf2{0.f, 0.f}, vf2{0.f, 0.f}, vf2{0.f, 0.f}, vf2{0.f, 0.f}};
#pragma unroll
    for (int i = 0; i < KQ / 2; ++i) {
      const vf2 h2v = vf2{hv[i].x, hv[i].y};
#pragma unroll
      for (int j = 0; j < 4; ++j) pp[j] = __builtin_elementwise_fma(h2v, wv[j][i], pp[j]);
    }
    float pj[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      pj[j] = pp[j].x + pp[j].y;
      pj[j] += dpp_x1(pj[j]);
      pj[j] += dpp_x2(pj[j]);
    }
    float ig, fg, cg, og, av;
    if constexpr (A4) {
      ig = sigm(x4.x + pj[0]);
      fg = sigm(x4.y + pj[1]);
      cg = ftanh(x4.z + pj[2]);
      og = sigm(x4.w + pj[3]);
      av = q == 0 ? ig : q == 1 ? fg : q == 2 ? cg : og;
    } else {
      const float mine = q == 0 ? pj[0] : q == 1 ? pj[1] : q == 2 ? pj[2] : pj[3];
      const float pre = xacc + mine;
      av = q == 2 ? ftanh(pre) : sigm(pre);
      ig = quad_bcast<0>(av); fg = quad_bcast<1>(av);
      cg = quad_bcast<2>(av); og = quad_bcast<3>(av);
    }
    const float c = fg * creg + ig * cg;
    const float h = og * ftanh(c);
    creg = c;
    if (act && q == 0) hn[u] = h;
    ph = h; pc = c; pav = av;
    __syncthreads();
  }
  LSTM_TICK(3);                                  // the step loop
  if (a.S > 0 && act) {
    if (q == 0) {
      hb[0] = ph;
      if (cb && a.S - 1 < keepS) cb[0] = pc;
    }
    if (gp && a.S - 1 < keepS) gp[0] = pav;
  }
}

// BR: rows of W_hh per lane of a 16-lane row (16 BR >= 4H); the body is
// lstm_bwd_q_body (lstm_cell.hpp), shared with the BPTT + weight-gradient
// launch of linear_kernels.hip
template <int BR, bool STG>
__global__ void __launch_bounds__(kVT)
lstm_bwd_q_kernel(LstmBwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) float bstage[];
  LSTM_T0();
  lstm_bwd_q_body<BR, SMI_BPTT_CH4 != 0, STG>(a, blockIdx.x, bstage);
  LSTM_TICK(4);                                  // the whole BPTT (its own launch)
}
#endif  // SMI_LSTM_VALU_HALF

// VALU recurrence selection: SMI_LSTM_VALU = 0 (never), 1 (always when the
// shape fits), unset: when the batch leaves at least one segment group per CU
// idle under the MFMA forms (B <= 2 x CUs, i.e. R <= 2)
static int lstm_valu_mode() {
  static int m = -2;
  if (m == -2) {
    const char* e = getenv("SMI_LSTM_VALU");
    m = e ? atoi(e) : -1;
  }
  return m;
}
static int device_cus() {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
      cus = 256;
  }
  return cus;
}
// segments per workgroup of the VALU forms, 0 = use the MFMA forms
static int lstm_valu_r(int B, int H) {
  if (H < 1 || H > 128) return 0;
  const int m = lstm_valu_mode();
  if (m == 0) return 0;
  static const int force_r = [] {                 // SMI_LSTM_VALU_R = 1 | 2 | 4: A/B knob
    const char* e = getenv("SMI_LSTM_VALU_R");
    const int r = e ? atoi(e) : 0;
    return (r == 1 || r == 2 || r == 4) ? r : 0;
  }();
  if (force_r) return force_r;
  const int cus = device_cus();
  int R = (B + cus - 1) / cus;
  if (R < 1) R = 1;
  if (R == 3) R = 4;
  if (R > 4) return 0;
  // auto: the row forms only at one segment per CU (the K-split q form); at
  // two or more the r4 MFMA form (384 / 512 segments: 4.32 / 4.98 ms per
  // learn against 4.76 / 5.44 with R = 2 and 4.42 / 5.12 with the q form at
  // two workgroups per CU, round 6, profiles/r06/ab/lstm_form_*)
  if (m < 0 && R > 1) return 0;
  return R;
}

// LDS of the staged x sequence and the precomputed x parts (KX > 0); the fused
// form is used up to kVxMax (S <= 52 steps at H = 100, x width <= 64)
[[maybe_unused]] constexpr size_t kVxMax = 120 * 1024;
static size_t lstm_fwd_v_lds(int S, int R, int KX, int blk) {
  return ((((size_t)S * R * KX + 3) & ~(size_t)3) + (size_t)S * R * blk) * 4;
}
#if SMI_LSTM_VALU_HALF
template <int R, int KX>
static void fwd_v_dispatch_kp(const LstmFwdArgs& a, hipStream_t st) {
  const dim3 grid((a.B + R - 1) / R), blk((4 * a.H + 63) & ~63);
  const size_t lds = KX > 0 ? lstm_fwd_v_lds(a.S, R, KX, blk.x) : 0;
#define SMI_FV(KP)                                                                 \
  do {                                                                             \
    allow_lds(lstm_fwd_v_kernel<R, KP, KX>, lds);                                  \
    hipLaunchKernelGGL((lstm_fwd_v_kernel<R, KP, KX>), grid, blk, lds, st, a);     \
  } while (0)
  if (a.H <= 64) SMI_FV(64);
  else if (a.H <= 104) SMI_FV(104);
  else SMI_FV(128);
#undef SMI_FV
}
// x W_ih^T fused only at R = 1 (its W_ih row joins the W_hh row in registers:
// at R >= 2 the two segments' operands no longer fit next to them); R >= 2
// reads the xproj GEMM's output (launch_lstm_fwd_x returns SMI_E_NOFIT)
static void fwd_v_dispatch(const LstmFwdArgs& a, int R, hipStream_t st) {
  if (R == 1) fwd_v_dispatch_kp<1, 0>(a, st);
  else if (R == 2) fwd_v_dispatch_kp<2, 0>(a, st);
  else fwd_v_dispatch_kp<4, 0>(a, st);
}
template <int R>
static void bwd_v_dispatch_kp(const LstmBwdArgs& a, hipStream_t st) {
  const dim3 grid((a.B + R - 1) / R), blk((4 * a.H + 63) & ~63);
  if (a.H <= 64) hipLaunchKernelGGL((lstm_bwd_v_kernel<R, 64>), grid, blk, 0, st, a);
  else if (a.H <= 104) hipLaunchKernelGGL((lstm_bwd_v_kernel<R, 104>), grid, blk, 0, st, a);
  else hipLaunchKernelGGL((lstm_bwd_v_kernel<R, 128>), grid, blk, 0, st, a);
}

// the VALU forms' entry points for the launchers (the other half of the file
// when it is compiled in two parts): kx 0 = xproj input, else the fused x
// projection at R = 1 with x widths <= kx (48 / 64)
// the K-split forms at one segment per workgroup (SMI_LSTM_Q=0: the R = 1
// row forms instead; A/B knob)
static bool use_q() {
  static const bool on = [] { const char* e = getenv("SMI_LSTM_Q"); return !(e && e[0] == '0'); }();
  return on;
}
bool lstm_use_q() { return use_q(); }
// x parts on the matrix cores (SMI_LSTM_XM=0: the VALU K-split form; A/B knob)
static bool use_xm() {
  static const bool on = [] { const char* e = getenv("SMI_LSTM_XM"); return !(e && e[0] == '0'); }();
  return on;
}
// a1 (optional): the second sequence set of a dual launch (same H / x width)
template <int XQ>
static void fwd_q_dispatch(const LstmFwdArgs& a, hipStream_t st, const LstmFwdArgs* a1 = nullptr) {
  const dim3 grid(a.B + (a1 ? a1->B : 0)), blk((4 * a.H + 63) & ~63);
  const LstmFwdArgs& a2 = a1 ? *a1 : a;
  const int smax = a1 && a1->S > a.S ? a1->S : a.S;
  auto aligned = [&](const float* LstmFwdArgs::*p, uintptr_t m) {
    return (reinterpret_cast<uintptr_t>(a.*p) & m) == 0 && (reinterpret_cast<uintptr_t>(a2.*p) & m) == 0;
  };
  // the matrix-core x parts load W_ih rows as float2 runs
  const bool xm = XQ > 0 && use_xm() && a.din % 2 == 0 && aligned(&LstmFwdArgs::w_ih, 7);
  // W_hh register layout (SMI_LSTM_WI; A/B knob): 0 a contiguous quarter row
  // per lane, 1 k pairs interleaved over the quad (float2 loads), 2 float4 runs
  // interleaved (float4 loads); a shape / alignment the vector loads cannot
  // take steps down (the kernel has no run-time vector / scalar branch)
  static const int wi_knob = [] { const char* e = getenv("SMI_LSTM_WI"); return e && e[0] ? atoi(e) : 2; }();
  int wi = wi_knob;
  if (wi == 2 && !(a.H % 4 == 0 && aligned(&LstmFwdArgs::w_hh, 15))) wi = 1;
  if (wi == 1 && !(a.H % 2 == 0 && aligned(&LstmFwdArgs::w_hh, 7))) wi = 0;
  // all four gates finished in every lane (SMI_LSTM_A4=0: one gate per lane +
  // quad broadcasts; A/B knob)
  static const bool a4 = [] { const char* e = getenv("SMI_LSTM_A4"); return !(e && e[0] == '0'); }();
  const size_t lds = XQ > 0 ? lstm_fwd_v_lds(smax, 1, 4 * XQ, blk.x) : 0;
#define SMI_FQ(KQ, W)                                                              \
  do {                                                                             \
    if (xm && a4) {                                                                \
      allow_lds(lstm_fwd_q_kernel<KQ, XQ, true, W, XQ != 0>, lds);                 \
      hipLaunchKernelGGL((lstm_fwd_q_kernel<KQ, XQ, true, W, XQ != 0>), grid, blk, lds, st, a, a2); \
    } else if (xm) {                                                               \
      allow_lds(lstm_fwd_q_kernel<KQ, XQ, true, W>, lds);                          \
      hipLaunchKernelGGL((lstm_fwd_q_kernel<KQ, XQ, true, W>), grid, blk, lds, st, a, a2);  \
    } else {                                                                       \
      allow_lds(lstm_fwd_q_kernel<KQ, XQ, false, W>, lds);                         \
      hipLaunchKernelGGL((lstm_fwd_q_kernel<KQ, XQ, false, W>), grid, blk, lds, st, a, a2); \
    }                                                                              \
  } while (0)
  if (a.H <= 64) {
    if (wi == 2) SMI_FQ(16, 2);
    else if (wi == 1) SMI_FQ(16, 1);
    else SMI_FQ(16, 0);
  } else if (a.H <= 112 && wi == 2) {
    SMI_FQ(28, 2);
  } else if (a.H <= 104) {
    if (wi == 1) SMI_FQ(26, 1);
    else SMI_FQ(26, 0);
  } else {
    if (wi == 2) SMI_FQ(32, 2);
    else if (wi == 1) SMI_FQ(32, 1);
    else SMI_FQ(32, 0);
  }
#undef SMI_FQ
}
// two sequence sets in one launch, one segment per workgroup (fused x parts)
void lstm_q_fwd_dual(const LstmFwdArgs& a, const LstmFwdArgs& a1, int kx, hipStream_t st) {
  if (kx <= 48) fwd_q_dispatch<12>(a, st, &a1);
  else fwd_q_dispatch<16>(a, st, &a1);
}
void lstm_v_fwd(const LstmFwdArgs& a, int R, int kx, hipStream_t st) {
  if (R == 1 && use_q()) {
    if (kx == 0) fwd_q_dispatch<0>(a, st);
    else if (kx <= 48) fwd_q_dispatch<12>(a, st);
    else fwd_q_dispatch<16>(a, st);
    return;
  }
  if (kx == 0) fwd_v_dispatch(a, R, st);
  else if (kx <= 48) fwd_v_dispatch_kp<1, 48>(a, st);
  else fwd_v_dispatch_kp<1, 64>(a, st);
}
// the BPTT's step inputs staged in LDS (SMI_BWD_STAGE=1; A/B knob, off: the
// staging prologue cost what the loop's per-step vmcnt(0) did -- 128 segments
// 2.771-2.777 vs 2.764-2.765 ms per learn, BPTT 27.7 vs 26.7-27.0 us at 256,
// profiles/r06/ab/bwd_stage_*; the inputs are read two steps ahead instead)
bool use_bwd_stage() {
  static const bool on = [] { const char* e = getenv("SMI_BWD_STAGE"); return e && e[0] == '1'; }();
  return on;
}
// the BPTT's K-split form loads W_hh as float4 runs (lstm_bwd_q_body)
bool lstm_bwd_q_ok(int H, const float* w_hh) {
  return use_q() && H % 4 == 0 && (reinterpret_cast<uintptr_t>(w_hh) & 15) == 0;
}
void lstm_v_bwd(const LstmBwdArgs& a, int R, hipStream_t st) {
  if (R == 1 && lstm_bwd_q_ok(a.H, a.w_hh)) {
    const dim3 grid(a.B), blk((4 * a.H + 63) & ~63);
    // the step inputs staged in LDS when they fit (lstm_bwd_q_body)
    const size_t stg = (size_t)lstm_bwd_stage_floats(a.S, a.H) * 4;
    const bool s = use_bwd_stage() && stg <= kBwdStageMax;
#define SMI_BQ(BR_)                                                                       \
    do {                                                                                  \
      if (s) {                                                                            \
        allow_lds(lstm_bwd_q_kernel<BR_, true>, stg);                                     \
        hipLaunchKernelGGL((lstm_bwd_q_kernel<BR_, true>), grid, blk, stg, st, a);        \
      } else {                                                                            \
        hipLaunchKernelGGL((lstm_bwd_q_kernel<BR_, false>), grid, blk, 0, st, a);         \
      }                                                                                   \
    } while (0)
    if (a.H <= 64) SMI_BQ(16);
    else if (a.H <= 100) SMI_BQ(25);
    else SMI_BQ(32);
#undef SMI_BQ
    return;
  }
  if (R == 1) bwd_v_dispatch_kp<1>(a, st);
  else if (R == 2) bwd_v_dispatch_kp<2>(a, st);
  else bwd_v_dispatch_kp<4>(a, st);
}
#ifdef SMI_PROF
// the VALU half's phase ticks (its own copy of g_lstm_ticks when the file is
// compiled in two parts)
extern "C" int smi_lstm_v_phase_ticks(unsigned long long* out /* [8] */) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_lstm_ticks), sizeof(g_lstm_ticks)) != hipSuccess)
    return SMI_E_LAUNCH;
  static const unsigned long long zero[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  return hipMemcpyToSymbol(HIP_SYMBOL(g_lstm_ticks), zero, sizeof(zero)) == hipSuccess ? SMI_OK
                                                                                        : SMI_E_LAUNCH;
}
#endif
#else
void lstm_v_fwd(const LstmFwdArgs& a, int R, int kx, hipStream_t st);
void lstm_v_bwd(const LstmBwdArgs& a, int R, hipStream_t st);
void lstm_q_fwd_dual(const LstmFwdArgs& a, const LstmFwdArgs& a1, int kx, hipStream_t st);
#endif  // SMI_LSTM_VALU_HALF

#if SMI_LSTM_MFMA
static int use_r4() {
  static int u = -1;
  if (u < 0) {
    const char* e = getenv("SMI_LSTM_R4");
    u = (e && e[0] == '0') ? 0 : 1;
  }
  return u;
}

#ifdef SMI_PROF
extern "C" int smi_lstm_phase_ticks(unsigned long long* out /* [8] */) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_lstm_ticks), sizeof(g_lstm_ticks)) != hipSuccess)
    return SMI_E_LAUNCH;
  static const unsigned long long zero[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  return hipMemcpyToSymbol(HIP_SYMBOL(g_lstm_ticks), zero, sizeof(zero)) == hipSuccess ? SMI_OK
                                                                                        : SMI_E_LAUNCH;
}
#endif

int64_t lstm_fwd_lds(int H) { return (int64_t)2 * LR * lstm_ld(4 * lstm_q(H)) * 4; }
int64_t lstm_bwd_lds(int H) { return (int64_t)2 * LR * lstm_ld(4 * H) * 4; }

// the r4 forward's fixed-width row loads (VF): W_hh float4 runs, W_ih float2
// runs (SMI_R4_VF=0: the alignment-branching loads; A/B knob)
static bool r4_vf(const LstmFwdArgs& a, bool fused_x) {
  static const bool on = [] { const char* e = getenv("SMI_R4_VF"); return !(e && e[0] == '0'); }();
  auto al = [](const void* p, uintptr_t m) { return (reinterpret_cast<uintptr_t>(p) & m) == 0; };
  if (!on || a.H % 4 != 0 || !al(a.w_hh, 15)) return false;
  return !fused_x || (a.din % 2 == 0 && a.din >= 2 && al(a.w_ih, 7));
}

// the r4 forward's weight staging (lstm_fwd_r4_kernel): dynamic LDS bytes, 0
// when it does not apply (off unless SMI_R4_WSTAGE=1: measured slower, the
// prologue 11.1 -> 18.8 us and C3 6.92-6.93 -> 7.15-7.19 ms per learn -- three
// staged passes with their barriers and 4-way conflicted row reads cost more
// than the row-per-lane loads; also: more than one resident round of
// workgroups, rows not in float4 runs, a pass beyond one trip)
static size_t r4_wstage_bytes(const LstmFwdArgs& a, bool fused_x) {
  static const bool on = [] { const char* e = getenv("SMI_R4_WSTAGE"); return e && e[0] == '1'; }();
  if (!on) return 0;
  const int H = a.H, G4 = 4 * H;
  auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  if ((a.B + LR4 - 1) / LR4 > device_cus() || H % 4 != 0 || !al16(a.w_hh)) return 0;
  const int64_t cap4 = (int64_t)R4_PT * kWG8;
  int64_t floats = 2LL * H * H;                    // half of W_hh per pass
  if (floats / 4 > cap4) return 0;
  if (fused_x) {
    if (!al16(a.w_ih) || ((int64_t)G4 * a.din) % 4 != 0 || (int64_t)G4 * a.din / 4 > cap4) return 0;
    floats = std::max<int64_t>(floats, (int64_t)G4 * a.din);
  }
  return (size_t)floats * 4;
}

int launch_lstm_fwd(const float* xproj, const float* w_hh, const float* b_hh, const float* h0,
                    const float* c0, int S, int B, int H, float* hbuf, float* cbuf, float* gates,
                    hipStream_t st, const int* skip, int keep) {
  if (B <= 0 || S < 0) return SMI_OK;
  if (H < 1 || H > 256) return set_error(SMI_E_ARG, "lstm: hidden size must be in [1, 256]");
  LstmFwdArgs a{xproj, w_hh, b_hh, h0, c0, S, B, H, hbuf, cbuf, gates, skip};
  a.keep = keep;
  const int kslot = ktime_begin(st);
  // algorithmic flops: the recurrent GEMM h W_hh^T of every step
  struct End { int s; hipStream_t st; double f;
               ~End() { ktime_end(s, KT_LSTM_FWD, f, st); } } end_{kslot, st, 8.0 * B * H * (double)H * S};
  if (const int R = lstm_valu_r(B, H)) {
    lstm_v_fwd(a, R, 0, st);
    return check_launch("lstm_fwd_v_kernel");
  }
  if (H <= 128 && use_r4()) {
    const dim3 g4((B + LR4 - 1) / LR4);
    const size_t wl = r4_wstage_bytes(a, false);
    a.wstage = wl > 0;
    const bool vf = !a.wstage && r4_vf(a, false);
#define SMI_R4F(KP_)                                                                        \
    do {                                                                                    \
      if (vf) {                                                                             \
        hipLaunchKernelGGL((lstm_fwd_r4_kernel<KP_, 0, true>), g4, dim3(kWG8), 0, st, a);   \
      } else {                                                                              \
        if (wl) allow_lds(lstm_fwd_r4_kernel<KP_, 0>, wl);                                  \
        hipLaunchKernelGGL((lstm_fwd_r4_kernel<KP_, 0>), g4, dim3(kWG8), wl, st, a);        \
      }                                                                                     \
    } while (0)
    if (H <= 32) SMI_R4F(32);
    else if (H <= 64) SMI_R4F(64);
    else if (H <= 104) SMI_R4F(104);
    else SMI_R4F(128);
#undef SMI_R4F
    return check_launch("lstm_fwd_r4_kernel");
  }
  const size_t lds = (size_t)lstm_fwd_lds(H);
  const dim3 grid((B + LR - 1) / LR);
  if (H <= 64) {
    const size_t l16 = (size_t)2 * LR * lstm_ld(4 * 16) * 4;
    allow_lds(lstm_fwd_reg_kernel<16>, l16);
    hipLaunchKernelGGL(lstm_fwd_reg_kernel<16>, grid, dim3(kWG8), l16, st, a);
    return check_launch("lstm_fwd_reg_kernel");
  }
  if (H <= 112) {                      // the reference default H = 100: 112 W regs/lane
    const size_t l28 = (size_t)2 * LR * lstm_ld(4 * 28) * 4;
    allow_lds(lstm_fwd_reg_kernel<28>, l28);
    hipLaunchKernelGGL(lstm_fwd_reg_kernel<28>, grid, dim3(kWG8), l28, st, a);
    return check_launch("lstm_fwd_reg_kernel");
  }
  const int nut = (H + 15) / 16;
  if (nut <= 4) {
    allow_lds(lstm_fwd_kernel<1>, lds);
    hipLaunchKernelGGL(lstm_fwd_kernel<1>, grid, dim3(kWG), lds, st, a);
  } else if (nut <= 8) {
    allow_lds(lstm_fwd_kernel<2>, lds);
    hipLaunchKernelGGL(lstm_fwd_kernel<2>, grid, dim3(kWG), lds, st, a);
  } else {
    allow_lds(lstm_fwd_kernel<4>, lds);
    hipLaunchKernelGGL(lstm_fwd_kernel<4>, grid, dim3(kWG), lds, st, a);
  }
  return check_launch("lstm_fwd_kernel");
}

// LSTM forward with the input projection fused (din <= 64, H <= 104): returns
// SMI_E_NOFIT when the shape needs the xproj GEMM + launch_lstm_fwd instead
int launch_lstm_fwd_x(const float* x, int64_t ldx, int din, const float* w_ih, const float* b_ih,
                      const float* w_hh, const float* b_hh, const float* h0, const float* c0,
                      int S, int B, int H, float* hbuf, float* cbuf, float* gates,
                      hipStream_t st, const int* skip, int keep) {
  if (!use_r4() || din < 1 || din > 64 || H < 1 || H > 104) return SMI_E_NOFIT;
  if (B <= 0 || S < 0) return SMI_OK;
  const int R = lstm_valu_r(B, H);
  if (R > 1) return SMI_E_NOFIT;                 // xproj GEMM + the VALU recurrence
  if (R == 1 && lstm_fwd_v_lds(S, 1, din <= 48 ? 48 : 64, (4 * H + 63) & ~63) > kVxMax)
    return SMI_E_NOFIT;                            // staged x + x parts > the LDS budget
  LstmFwdArgs a{nullptr, w_hh, b_hh, h0, c0, S, B, H, hbuf, cbuf, gates, skip,
                x, ldx, din, w_ih, b_ih, keep};
  const int kslot = ktime_begin(st);
  struct End { int s; hipStream_t st; double f;
               ~End() { ktime_end(s, KT_LSTM_FWD, f, st); } } end_{
      kslot, st, 8.0 * B * H * (double)(H + din) * S};
  if (R == 1) {
    lstm_v_fwd(a, 1, din <= 48 ? 48 : 64, st);
    return check_launch("lstm_fwd_v_kernel");
  }
  const dim3 g4((B + LR4 - 1) / LR4);
  const size_t wl = r4_wstage_bytes(a, true);
  a.wstage = wl > 0;
  const bool vf = !a.wstage && r4_vf(a, true);
#define SMI_R4X(KP_, KX_)                                                                     \
  do {                                                                                        \
    if (vf) {                                                                                 \
      hipLaunchKernelGGL((lstm_fwd_r4_kernel<KP_, KX_, true>), g4, dim3(kWG8), 0, st, a);     \
    } else {                                                                                  \
      if (wl) allow_lds(lstm_fwd_r4_kernel<KP_, KX_>, wl);                                    \
      hipLaunchKernelGGL((lstm_fwd_r4_kernel<KP_, KX_>), g4, dim3(kWG8), wl, st, a);          \
    }                                                                                         \
  } while (0)
  if (din <= 48) {
    if (H <= 64) SMI_R4X(64, 48);
    else SMI_R4X(104, 48);
  } else {
    if (H <= 64) SMI_R4X(64, 64);
    else SMI_R4X(104, 64);
  }
#undef SMI_R4X
  return check_launch("lstm_fwd_r4_kernel");
}

bool lstm_use_q();
// BR of the BPTT's one-segment-per-workgroup K-split form (lstm_bwd_q_kernel)
// when launch_lstm_bwd would run it for (B, H), else 0: the form that the
// BPTT + weight-gradient launch (linear_kernels.hip) embeds
bool lstm_bwd_q_ok(int H, const float* w_hh);
int lstm_bwd_q_form(int B, int H, const float* w_hh) {
  if (lstm_valu_r(B, H) != 1 || !lstm_bwd_q_ok(H, w_hh)) return 0;
  return H <= 64 ? 16 : H <= 100 ? 25 : 32;
}

// two independent fused-input forwards (same H and input width, e.g. the GAE
// critic pass and the reference policy's forward) in ONE launch at one segment
// per workgroup (the K-split form): SMI_E_NOFIT when that form does not run
// for B0 + B1 segments on this device or the widths differ
bool lstm_fwd_x_dual_fits(int B0, int B1, int S, int H, int din) {
  if (!use_r4() || !lstm_use_q() || din < 1 || din > 64 || H < 1 || H > 104 || B0 <= 0 || B1 <= 0)
    return false;
  if (lstm_valu_r(B0 + B1, H) != 1) return false;
  return lstm_fwd_v_lds(S, 1, din <= 48 ? 48 : 64, (4 * H + 63) & ~63) <= kVxMax;
}

int launch_lstm_fwd_x_dual(const LstmFwdArgs& a0, const LstmFwdArgs& a1, hipStream_t st) {
  const int H = a0.H, din = a0.din;
  const int smax = a0.S > a1.S ? a0.S : a1.S;
  if (a0.H != a1.H || a0.din != a1.din || !lstm_fwd_x_dual_fits(a0.B, a1.B, smax, H, din))
    return SMI_E_NOFIT;
  const int kx = din <= 48 ? 48 : 64;
  const int kslot = ktime_begin(st);
  lstm_q_fwd_dual(a0, a1, kx, st);
  ktime_end(kslot, KT_LSTM_FWD,
            8.0 * H * (double)(H + din) * ((double)a0.B * a0.S + (double)a1.B * a1.S), st);
  return check_launch("lstm_fwd_q_kernel");
}

int launch_lstm_bwd(const float* dh, const float* gates, const float* cbuf, const float* w_hh,
                    int S, int B, int H, float* dgates, hipStream_t st, const int* skip) {
  if (B <= 0 || S <= 0) return SMI_OK;
  if (H < 1 || H > 256) return set_error(SMI_E_ARG, "lstm: hidden size must be in [1, 256]");
  LstmBwdArgs a{dh, gates, cbuf, w_hh, S, B, H, dgates, skip};
  const int kslot = ktime_begin(st);
  struct End { int s; hipStream_t st; double f;
               ~End() { ktime_end(s, KT_LSTM_BWD, f, st); } } end_{kslot, st,
                                                                 8.0 * B * H * (double)H * (S - 1)};
  if (const int R = lstm_valu_r(B, H)) {
    lstm_v_bwd(a, R, st);
    return check_launch("lstm_bwd_v_kernel");
  }
  if (H <= 128 && use_r4()) {
    const int nu = (H + 63) / 64, wpg = 8 / nu;
    const int kw = (4 * H + wpg - 1) / wpg;
    const dim3 g4((B + LR4 - 1) / LR4);
    if (kw <= 32) hipLaunchKernelGGL(lstm_bwd_r4_kernel<32>, g4, dim3(kWG8), 0, st, a);
    else if (kw <= 64) hipLaunchKernelGGL(lstm_bwd_r4_kernel<64>, g4, dim3(kWG8), 0, st, a);
    else if (kw <= 104) hipLaunchKernelGGL(lstm_bwd_r4_kernel<104>, g4, dim3(kWG8), 0, st, a);
    else hipLaunchKernelGGL(lstm_bwd_r4_kernel<128>, g4, dim3(kWG8), 0, st, a);
    return check_launch("lstm_bwd_r4_kernel");
  }
  const size_t lds = (size_t)lstm_bwd_lds(H);
  if (lds > 160 * 1024) return set_error(SMI_E_NOFIT, "lstm: hidden size too large for LDS");
  const dim3 grid((B + LR - 1) / LR);
  if (H == 64) {
    allow_lds(lstm_bwd_reg_kernel<64>, lds);
    hipLaunchKernelGGL(lstm_bwd_reg_kernel<64>, grid, dim3(kWG8), lds, st, a);
    return check_launch("lstm_bwd_reg_kernel");
  }
  if (H == 100) {                      // the reference default: KS must equal H
    allow_lds(lstm_bwd_reg_kernel<100>, lds);
    hipLaunchKernelGGL(lstm_bwd_reg_kernel<100>, grid, dim3(kWG8), lds, st, a);
    return check_launch("lstm_bwd_reg_kernel");
  }
  const int nut = (H + 15) / 16;
  if (nut <= 4) {
    allow_lds(lstm_bwd_kernel<1>, lds);
    hipLaunchKernelGGL(lstm_bwd_kernel<1>, grid, dim3(kWG), lds, st, a);
  } else if (nut <= 8) {
    allow_lds(lstm_bwd_kernel<2>, lds);
    hipLaunchKernelGGL(lstm_bwd_kernel<2>, grid, dim3(kWG), lds, st, a);
  } else {
    allow_lds(lstm_bwd_kernel<4>, lds);
    hipLaunchKernelGGL(lstm_bwd_kernel<4>, grid, dim3(kWG), lds, st, a);
  }
  return check_launch("lstm_bwd_kernel");
}

#endif  // SMI_LSTM_MFMA

}  // namespace smi
