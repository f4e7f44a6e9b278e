// lstm_cell.hpp — LSTM cell arithmetic shared by the sequence kernels
// (lstm_kernels.hip) and the BPTT + weight-gradient launch (linear_kernels.hip):
// the activations, the kernel argument blocks, the lane-quad exchanges and the
// one-segment-per-workgroup BPTT body (lstm_bwd_q_body).
#pragma once
#include "smi_device.hpp"

namespace smi {

// Activations on the hardware transcendental units (v_exp_f32, v_rcp_f32: ~1
// ulp each).  sigmoid(x) = 1/(1 + 2^(-x log2 e)): a few ulp RELATIVE everywhere
// (no cancellation).  tanh must also be accurate RELATIVE to its value: the
// earlier 2 sigmoid(2x) - 1 form cancelled for small |x| (absolute error ~1e-7,
// i.e. 1e-4 relative at |x| ~ 1e-3), which made the LSTM outputs near zero
// ~1000x noisier than torch's and showed up as divergence from the fp64 oracle
// after 10 + 10 epochs (tests/test_gpu_parity_pinned.py).  Now: odd minimax
// polynomial for |x| < 0.625 (Cephes tanhf coefficients, ~2e-7 relative),
// 1 - 2/(e^{2|x|} + 1) beyond (no cancellation there: the result is >= 0.55).
// The libm forms cost ~4x the VALU issue slots and made the sequence kernels
// VALU-bound; these stay on the transcendental units plus ~6 FMAs.
__device__ __forceinline__ float sigm(float x) {
  return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(-1.4426950408889634f * x));
}
#ifdef SMI_OLD_TANH
__device__ __forceinline__ float ftanh(float x) { return 2.f * sigm(2.f * x) - 1.f; }
#else
__device__ __forceinline__ float ftanh(float x) {
  const float ax = fabsf(x);
  const float z = x * x;
  const float p = fmaf(fmaf(fmaf(fmaf(fmaf(-5.70498872745e-3f, z, 2.06390887954e-2f), z,
                                      -5.37397155531e-2f), z, 1.33314422036e-1f), z,
                            -3.33332819422e-1f), z * x, x);
  const float e = 1.f - 2.f * __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(2.8853900817779268f * ax));
  return ax < 0.625f ? p : copysignf(e, x);
}
#endif

struct LstmFwdArgs {
  const float* xproj;     // [S][B][4H] = x W_ih^T + b_ih
  const float* w_hh;      // [4H][H]
  const float* b_hh;      // [4H]
  const float* h0;        // [B][H]
  const float* c0;        // [B][H]
  int S, B, H;
  float* hbuf;            // [S+1][B][H]
  float* cbuf;            // [S+1][B][H] or null
  float* gates;           // [S][B][4H] activated, or null
  const int* skip;
  // fused input projection (lstm_fwd_r4_kernel<KP, KX > 0>): x_t W_ih^T + b_ih
  // inside the step instead of the xproj GEMM
  const float* x;         // [S][B][ldx]
  int64_t ldx;
  int din;
  const float* w_ih;      // [4H][din]
  const float* b_ih;      // [4H]
  // cbuf / gates are stored for steps t < keep only (0: all S steps): a forward
  // over more steps than a backward needs (the GAE critic pass over T + 1
  // steps serves as the first policy forward over its first E steps)
  int keep;
  // r4 MFMA forward (round 6): W_ih and W_hh reach the lanes' row registers
  // through LDS (coalesced global reads) instead of a row per lane from global
  // memory; set by the launcher with the dynamic LDS it sized for it
  int wstage;
};

struct LstmBwdArgs {
  const float* dh;        // [S][B][H]  dL/dh_t from the heads
  const float* gates;     // [S][B][4H] activated (i, f, g, o)
  const float* cbuf;      // [S+1][B][H]
  const float* w_hh;      // [4H][H]
  int S, B, H;
  float* dgates;          // [S][B][4H] dL/d(pre-activation gates)
  const int* skip;
};

typedef float vf2 __attribute__((ext_vector_type(2)));
constexpr int kVT = 512;      // threads of the VALU recurrence workgroups (4H <= 512)
template <int K>
__device__ __forceinline__ float quad_bcast(float v) {      // lane K of each quad
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), K * 0x55, 0xF, 0xF, false));
}

__device__ __forceinline__ float dpp_x1(float v) {            // quad lane l ^ 1
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false));
}
__device__ __forceinline__ float dpp_x2(float v) {            // quad lane l ^ 2
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, false));
}
__device__ __forceinline__ float dpp_hmirror(float v) {       // row_half_mirror
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x141, 0xF, 0xF, false));
}
__device__ __forceinline__ float dpp_ror8(float v) {          // row_ror:8
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x128, 0xF, 0xF, false));
}

// BPTT of one segment (b) at one segment per workgroup (the K-split form,
// lstm_kernels.hip): BR rows of W_hh per lane of a 16-lane row (16 BR >= 4H),
// BRP their padding to whole b128 reads
// CH4: the recurrent dot product in four FMA chains instead of two (build
// knob SMI_BPTT_CH4, default on; variant 'ch2' of surreal_amd/build.py is the
// round-5 form: 128 segments 2.919 vs 2.908 ms per learn, interleaved pairs)
#ifndef SMI_BPTT_CH4
#define SMI_BPTT_CH4 1
#endif
// Floats of the BPTT's staged per-step inputs (lstm_bwd_q_body with a
// stage): gates [S][4H], cell states [S+1][H], dh [S][H] of one segment
__host__ __device__ inline int64_t lstm_bwd_stage_floats(int S, int H) {
  return (int64_t)S * 4 * H + (int64_t)(S + 1) * H + (int64_t)S * H;
}

// STG: stage = LDS of lstm_bwd_stage_floats(S, H) floats, 16-byte aligned
// (a compile-time choice: a run-time one leaves the global-load path's waits
// in the loop).  With it every step input (activated gates, c_t, c_{t-1}, dh_t) is
// copied to LDS in the prologue and the step loop issues no global load
// (without it the loop header waits vmcnt(0) every step: the inputs fetched
// two steps ahead, and the previous step's dgates store, stores counting in
// vmcnt on gfx950).  Measured neutral-to-worse (the staging prologue costs
// what the waits did): an A/B knob, SMI_BWD_STAGE=1 (round 6)
template <int BR, bool CH4 = false, bool STG = false>
__device__ __forceinline__ void lstm_bwd_q_body(const LstmBwdArgs& a, int b,
                                                float* __restrict__ stage = nullptr) {
  if (a.skip && a.skip[0] != 0) return;
  constexpr int BRP = (BR + 3) & ~3;
  __shared__ __attribute__((aligned(16))) float dG[2][16 * BRP];
  const int H = a.H, B = a.B, G4 = 4 * H;
  const int tid = threadIdx.x, u = tid >> 2, q = tid & 3;
  const bool act = u < H;
  const int uc = act ? u : H - 1;
  const int g = q * H + uc;
  const int64_t BH = (int64_t)B * H;
  const int ug = tid >> 4, rr = tid & 15;
  for (int e = tid; e < 2 * 16 * BRP; e += blockDim.x) (&dG[0][0])[e] = 0.f;
  // W_hh[r][4ug + i], r in [rr*BR, rr*BR + BR)
  vf2 w01[BR], w23[BR];
  {
    // float4 loads (lstm_bwd_q_ok: H % 4 == 0 and a 16-byte aligned W_hh),
    // unconditional from clamped addresses with nothing selected on them: a
    // per-lane condition (or a run-time vector / scalar branch) turned the loads
    // into single dwords behind branches with a vmcnt(0) wait at each merge
    // (round 6).  Rows past 4H meet the zero padding of the dgates image; units
    // past H feed only lanes whose results are dropped.
    const int c0 = min(4 * ug, H - 4);
#pragma unroll
    for (int i = 0; i < BR; ++i) {
      const int r = min(rr * BR + i, G4 - 1);
      const float4 v = *reinterpret_cast<const float4*>(a.w_hh + (int64_t)r * H + c0);
      w01[i] = vf2{v.x, v.y};
      w23[i] = vf2{v.z, v.w};
    }
  }
  const int dgi = (g / BR) * BRP + g % BR;        // this lane's dgate in the padded image
  float gq, ct, ctm, dho, gqn, ctn, ctmn, dhon;
  if (a.S <= 0) return;
  float* sG = stage;                                // [S][4H]
  float* sC = STG ? sG + (int64_t)a.S * G4 : nullptr;       // [S+1][H]
  float* sD = STG ? sC + (int64_t)(a.S + 1) * H : nullptr;  // [S][H]
  if constexpr (STG) {
    // rows of 4H / H floats, float4 runs (H % 4 == 0: lstm_bwd_q_ok), eight
    // float4 loads per thread in flight per trip, then their LDS stores
    const int q4 = H >> 2, g4 = 4 * q4;
    const int ng = a.S * g4, nc = (a.S + 1) * q4, nd = a.S * q4;
    const int n4 = ng + nc + nd, NT = blockDim.x;
    auto src = [&](int e) -> const float4* {
      if (e < ng) {
        const int t = e / g4, j = e - t * g4;
        return reinterpret_cast<const float4*>(a.gates + ((int64_t)t * B + b) * G4) + j;
      }
      e -= ng;
      if (e < nc) {
        const int t = e / q4, j = e - t * q4;
        return reinterpret_cast<const float4*>(a.cbuf + (int64_t)t * BH + (int64_t)b * H) + j;
      }
      e -= nc;
      const int t = e / q4, j = e - t * q4;
      return reinterpret_cast<const float4*>(a.dh + (int64_t)t * BH + (int64_t)b * H) + j;
    };
    float4* s4 = reinterpret_cast<float4*>(stage);
    for (int e0 = tid; e0 < n4; e0 += 8 * NT) {
      float4 v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = *src(min(e0 + j * NT, n4 - 1));
#pragma unroll
      for (int j = 0; j < 8; ++j) s4[min(e0 + j * NT, n4 - 1)] = v[j];   // (a clamped index writes its owner's value)
    }
    __syncthreads();
  }
  auto fetch = [&](int t, float& G, float& C, float& CM, float& DH) {
    if constexpr (STG) {
      G = sG[t * G4 + g];
      C = sC[(t + 1) * H + uc];
      CM = sC[t * H + uc];
      DH = sD[t * H + uc];
    } else {
      G = a.gates[((int64_t)t * B + b) * G4 + g];
      C = a.cbuf[(int64_t)(t + 1) * BH + (int64_t)b * H + uc];
      CM = a.cbuf[(int64_t)t * BH + (int64_t)b * H + uc];
      DH = a.dh[(int64_t)t * BH + (int64_t)b * H + uc];
    }
  };
  fetch(a.S - 1, gq, ct, ctm, dho);
  fetch(a.S >= 2 ? a.S - 2 : 0, gqn, ctn, ctmn, dhon);
  float dcreg = 0.f, dhr = 0.f;
  __syncthreads();
  // waves past ceil(4H / 64) (the BPTT + dW launch's 512-thread workgroups:
  // an eighth wave at H = 100) hold only units past H and rows past 4H, whose
  // results are dropped: they take the step loop's barriers and nothing else
  // (one barrier per step, as below)
  if ((tid & ~63) >= ((G4 + 63) & ~63)) {
    for (int t = a.S - 1; t >= 0; --t) __syncthreads();
    return;
  }
  for (int t = a.S - 1; t >= 0; --t) {
    float* dgw = dG[t & 1];
    const float ig = quad_bcast<0>(gq), fg = quad_bcast<1>(gq);
    const float cg = quad_bcast<2>(gq), og = quad_bcast<3>(gq);
    const float dh = dho + dhr;
    const float tc = ftanh(ct);
    const float dc = dh * og * (1.f - tc * tc) + dcreg;
    const float d_o = (dh * tc) * (og * (1.f - og));
    const float d_i = (dc * cg) * (ig * (1.f - ig));
    const float d_g = (dc * ig) * (1.f - cg * cg);
    const float d_f = (dc * ctm) * (fg * (1.f - fg));
    dcreg = act ? dc * fg : 0.f;
    float dq = q == 0 ? d_i : q == 1 ? d_f : q == 2 ? d_g : d_o;
    dq = act ? dq : 0.f;
    if (act) {
      dgw[dgi] = dq;
      a.dgates[((int64_t)t * B + b) * G4 + g] = dq;
    }
    gq = gqn; ct = ctn; ctm = ctmn; dho = dhon;
    fetch(t >= 2 ? t - 2 : 0, gqn, ctn, ctmn, dhon);
    __syncthreads();
    if (t == 0) break;
    const float4* dp = reinterpret_cast<const float4*>(dgw + rr * BRP);
    float4 dv[BRP / 4];
#pragma unroll
    for (int i = 0; i < BRP / 4; ++i) dv[i] = dp[i];
    vf2 p01 = {0.f, 0.f}, p23 = {0.f, 0.f};
    if constexpr (CH4) {
      // four FMA chains (even / odd rows), half as long, summed at the end
      vf2 q01 = {0.f, 0.f}, q23 = {0.f, 0.f};
#pragma unroll
      for (int i = 0; i < BR; ++i) {
        const float d = (i & 3) == 0 ? dv[i >> 2].x : (i & 3) == 1 ? dv[i >> 2].y
                      : (i & 3) == 2 ? dv[i >> 2].z : dv[i >> 2].w;
        if (i & 1) {
          q01 = __builtin_elementwise_fma(vf2{d, d}, w01[i], q01);
          q23 = __builtin_elementwise_fma(vf2{d, d}, w23[i], q23);
        } else {
          p01 = __builtin_elementwise_fma(vf2{d, d}, w01[i], p01);
          p23 = __builtin_elementwise_fma(vf2{d, d}, w23[i], p23);
        }
      }
      p01 = p01 + q01;
      p23 = p23 + q23;
    } else {
#pragma unroll
      for (int i = 0; i < BR; ++i) {
        const float d = (i & 3) == 0 ? dv[i >> 2].x : (i & 3) == 1 ? dv[i >> 2].y
                      : (i & 3) == 2 ? dv[i >> 2].z : dv[i >> 2].w;
        p01 = __builtin_elementwise_fma(vf2{d, d}, w01[i], p01);
        p23 = __builtin_elementwise_fma(vf2{d, d}, w23[i], p23);
      }
    }
    float pu[4] = {p01.x, p01.y, p23.x, p23.y};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      pu[k] += dpp_x1(pu[k]);
      pu[k] += dpp_x2(pu[k]);
      pu[k] += dpp_hmirror(pu[k]);
      pu[k] += dpp_ror8(pu[k]);
    }
    const int k = u & 3;                           // unit u = 4 ug + k
    dhr = k == 0 ? pu[0] : k == 1 ? pu[1] : k == 2 ? pu[2] : pu[3];
  }
}

}  // namespace smi
