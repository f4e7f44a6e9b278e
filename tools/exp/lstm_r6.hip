// Round 6: where the VALU LSTM step's time goes at one segment per workgroup
// (diagnostic only, not product code).  128 segments, H 100; the x part is
// the bias alone (the step loop is what is measured: per-step cost = the
// slope between S = 1 and S = 41, median of 30 launches each).
//   F0   the product forward step (lstm_fwd_q_kernel<28, ., ., 2>): thread
//        (u, q) = (tid >> 2, tid & 3) holds unit u's four gate rows over the k
//        runs 16 i + 4 q .. + 3; h_{t-1} read from LDS as 7 ds_read_b128 per
//        lane, packed FMAs, quad DPP sums; 512 threads
//   F1   F0 on 448 threads (7 waves: the 8th wave of F0 holds units 112-127,
//        none of them real at H = 100, and still runs the full step)
//   F2   row broadcast: lane = 16 q + i of wave w, unit u = 16 w + i, k in
//        [25 q, 25 q + 25): a lane reads TWO h values (one ds_read_b64 of a
//        permuted image) and the row's 16 lanes broadcast them to each other
//        with DPP row_newbcast (25 v_mov_dpp per step); gate pairs (0,1) and
//        (2,3) on v_pk_fma_f32 with the broadcast value in both halves; the
//        four rows' partials meet through ds_swizzle (xor 16) and ds_bpermute
//        (xor 32) in a fixed order; every lane then finishes all four gates
//   F0n / F0l  F0 without the FMAs (h reads summed) / without the LDS reads
//        (registers): subtractive diagnostics
//   hipcc -O3 --offload-arch=gfx950 -fno-slp-vectorize tools/exp/lstm_r6.hip -o /tmp/lstm_r6
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int H = 100, G4 = 400;
typedef float vf2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float sigm(float x) {
  return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(-1.4426950408889634f * x));
}
__device__ __forceinline__ float ftanh(float x) {
  const float ax = fabsf(x);
  const float z = x * x;
  const float p = fmaf(fmaf(fmaf(fmaf(fmaf(-5.70498872745e-3f, z, 2.06390887954e-2f), z,
                                      -5.37397155531e-2f), z, 1.33314422036e-1f), z,
                            -3.33332819422e-1f), z * x, x);
  const float e = 1.f - 2.f * __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(2.8853900817779268f * ax));
  return ax < 0.625f ? p : copysignf(e, x);
}
template <int K>
__device__ __forceinline__ float quad_bcast(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), K * 0x55, 0xF, 0xF, false));
}
__device__ __forceinline__ float dpp_x1(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false));
}
__device__ __forceinline__ float dpp_x2(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, false));
}
template <int N>
__device__ __forceinline__ float nbc(float v) {          // lane N of the row, to the whole row
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x150 + N, 0xF, 0xF, false));
}

struct Args {
  const float* w_hh; const float* b_ih; const float* b_hh; const float* h0; const float* c0;
  int S, B;
  float* hbuf; float* cbuf; float* gates;
};

// ------------------------------------------------------------------ F0 / F1
// MODE 0: product step; 1: no FMAs (h values summed); 2: no LDS reads
template <int NTH, int MODE>
__global__ void __launch_bounds__(512) f0_kernel(Args a) {
  constexpr int KQ = 28;
  __shared__ __attribute__((aligned(16))) float hS[2][4 * KQ];
  const int B = a.B, b = blockIdx.x;
  const int tid = threadIdx.x, u = tid >> 2, q = tid & 3;
  const bool act = u < H;
  const int uc = act ? u : H - 1;
  const int g = q * H + uc;
  const int64_t BH = (int64_t)B * H;
  const float bh = a.b_hh[g] + a.b_ih[g];
  float creg = a.c0[(int64_t)b * H + uc];
  if (act && q == 0) a.cbuf[(int64_t)b * H + u] = creg;
  for (int e = tid; e < 4 * KQ; e += NTH) {
    const float v = e < H ? a.h0[(int64_t)b * H + e] : 0.f;
    hS[0][e] = v;
    hS[1][e] = 0.f;
    if (e < H) a.hbuf[(int64_t)b * H + e] = v;
  }
  vf2 wv[4][KQ / 2];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float* r = a.w_hh + (int64_t)(j * H + uc) * H;
#pragma unroll
    for (int i = 0; i < KQ / 4; ++i) {
      const int k = 16 * i + 4 * q;
      const float4 v = k + 3 < H ? *reinterpret_cast<const float4*>(r + k) : float4{0.f, 0.f, 0.f, 0.f};
      wv[j][2 * i] = vf2{v.x, v.y};
      wv[j][2 * i + 1] = vf2{v.z, v.w};
    }
  }
  __syncthreads();
  float* hb = a.hbuf + BH + (int64_t)b * H + uc;
  float* cb = a.cbuf + BH + (int64_t)b * H + uc;
  float* gp = a.gates + (int64_t)b * G4 + g;
  const int64_t gstep = (int64_t)B * G4;
  float ph = 0.f, pc = 0.f, pav = 0.f;
  float regh = 0.f;
  for (int t = 0; t < a.S; ++t) {
    const float* hp = hS[t & 1] + 4 * q;
    float* hn = hS[(t + 1) & 1];
    float2 hv[KQ / 2];
    if (MODE == 2) {
#pragma unroll
      for (int i = 0; i < KQ / 2; ++i) hv[i] = float2{regh + 0.01f * i, regh - 0.02f * i};
    } else {
      const float4* h4 = reinterpret_cast<const float4*>(hp);
#pragma unroll
      for (int i = 0; i < KQ / 4; ++i) {
        const float4 v = h4[4 * i];
        hv[2 * i] = float2{v.x, v.y};
        hv[2 * i + 1] = float2{v.z, v.w};
      }
    }
    if (t > 0 && act) {
      if (q == 0) {
        hb[0] = ph; hb += BH;
        cb[0] = pc; cb += BH;
      }
      gp[0] = pav; gp += gstep;
    }
    float pj[4];
    if (MODE == 1) {
      float s = 0.f;
#pragma unroll
      for (int i = 0; i < KQ / 2; ++i) s += hv[i].x + hv[i].y;
#pragma unroll
      for (int j = 0; j < 4; ++j) pj[j] = s * wv[j][0].x;
    } else {
      vf2 pp[4] = {vf2{0.f, 0.f}, vf2{0.f, 0.f}, vf2{0.f, 0.f}, vf2{0.f, 0.f}};
#pragma unroll
      for (int i = 0; i < KQ / 2; ++i) {
        const vf2 h2v = vf2{hv[i].x, hv[i].y};
#pragma unroll
        for (int j = 0; j < 4; ++j) pp[j] = __builtin_elementwise_fma(h2v, wv[j][i], pp[j]);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) pj[j] = pp[j].x + pp[j].y;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      pj[j] += dpp_x1(pj[j]);
      pj[j] += dpp_x2(pj[j]);
    }
    const float mine = q == 0 ? pj[0] : q == 1 ? pj[1] : q == 2 ? pj[2] : pj[3];
    const float pre = bh + mine;
    const float av = q == 2 ? ftanh(pre) : sigm(pre);
    const float ig = quad_bcast<0>(av), fg = quad_bcast<1>(av);
    const float cg = quad_bcast<2>(av), og = quad_bcast<3>(av);
    const float c = fg * creg + ig * cg;
    const float h = og * ftanh(c);
    creg = c;
    regh = h;
    if (act && q == 0) hn[u] = h;
    ph = h; pc = c; pav = av;
    __syncthreads();
  }
  if (a.S > 0 && act) {
    if (q == 0) { hb[0] = ph; cb[0] = pc; }
    gp[0] = pav;
  }
}

// ------------------------------------------------------------------ F2
template <int N>
struct RowDot {
  // kk = 25 - N .. 24 of the (even / odd) chains
  static __device__ __forceinline__ void run(const vf2 (&hv2), const vf2 (&w01)[25], const vf2 (&w23)[25],
                                             vf2& a01e, vf2& a01o, vf2& a23e, vf2& a23o) {
    constexpr int kk = 25 - N;
    const float src = kk < 16 ? hv2.x : hv2.y;
    const float b = nbc<kk & 15>(src);
    const vf2 bb = vf2{b, b};
    if (kk & 1) {
      a01o = __builtin_elementwise_fma(bb, w01[kk], a01o);
      a23o = __builtin_elementwise_fma(bb, w23[kk], a23o);
    } else {
      a01e = __builtin_elementwise_fma(bb, w01[kk], a01e);
      a23e = __builtin_elementwise_fma(bb, w23[kk], a23e);
    }
    RowDot<N - 1>::run(hv2, w01, w23, a01e, a01o, a23e, a23o);
  }
};
template <>
struct RowDot<0> {
  static __device__ __forceinline__ void run(const vf2&, const vf2 (&)[25], const vf2 (&)[25], vf2&, vf2&,
                                             vf2&, vf2&) {}
};
__device__ __forceinline__ float xor16(float v) {   // lane ^ 16 (within 32-lane halves)
  return __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(v), (16 << 10) | 0x1F));
}
__device__ __forceinline__ float xor32(float v) {
  const int l = threadIdx.x & 63;
  return __int_as_float(__builtin_amdgcn_ds_bpermute((l ^ 32) << 2, __float_as_int(v)));
}
// h image: unit k's value at [(q*16 + (kk & 15)) * 2 + (kk >> 4)], q = k / 25, kk = k % 25
__device__ __forceinline__ int hpos(int k) {
  const int q = k / 25, kk = k - 25 * q;
  return ((q * 16 + (kk & 15)) << 1) + (kk >> 4);
}

__global__ void __launch_bounds__(448) f2_kernel(Args a) {
  constexpr int NTH = 448;
  __shared__ __attribute__((aligned(16))) float hP[2][128];
  const int B = a.B, b = blockIdx.x;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, q = l >> 4, i = l & 15;
  const int u = 16 * w + i;
  const bool act = u < H;
  const int uc = act ? u : H - 1;
  const int64_t BH = (int64_t)B * H;
  float bh4[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) bh4[j] = a.b_hh[j * H + uc] + a.b_ih[j * H + uc];
  float creg = a.c0[(int64_t)b * H + uc];
  if (act && q == 0) a.cbuf[(int64_t)b * H + u] = creg;
  for (int e = tid; e < 128; e += NTH) { hP[0][e] = 0.f; hP[1][e] = 0.f; }
  __syncthreads();
  for (int e = tid; e < H; e += NTH) {
    const float v = a.h0[(int64_t)b * H + e];
    hP[0][hpos(e)] = v;
    a.hbuf[(int64_t)b * H + e] = v;
  }
  vf2 w01[25], w23[25];
  {
    const float* r0 = a.w_hh + (int64_t)(0 * H + uc) * H + 25 * q;
    const float* r1 = a.w_hh + (int64_t)(1 * H + uc) * H + 25 * q;
    const float* r2 = a.w_hh + (int64_t)(2 * H + uc) * H + 25 * q;
    const float* r3 = a.w_hh + (int64_t)(3 * H + uc) * H + 25 * q;
#pragma unroll
    for (int kk = 0; kk < 25; ++kk) {
      w01[kk] = vf2{r0[kk], r1[kk]};
      w23[kk] = vf2{r2[kk], r3[kk]};
    }
  }
  __syncthreads();
  float* hb = a.hbuf + BH + (int64_t)b * H + uc;
  float* cb = a.cbuf + BH + (int64_t)b * H + uc;
  float* gp = a.gates + (int64_t)b * G4 + q * H + uc;
  const int64_t gstep = (int64_t)B * G4;
  const int hw = hpos(uc);
  float ph = 0.f, pc = 0.f, pav = 0.f;
  for (int t = 0; t < a.S; ++t) {
    const vf2 hv2 = *reinterpret_cast<const vf2*>(&hP[t & 1][2 * l]);
    float* hn = hP[(t + 1) & 1];
    if (t > 0 && act) {
      if (q == 0) {
        hb[0] = ph; hb += BH;
        cb[0] = pc; cb += BH;
      }
      gp[0] = pav; gp += gstep;
    }
    vf2 a01e = {0.f, 0.f}, a01o = {0.f, 0.f}, a23e = {0.f, 0.f}, a23o = {0.f, 0.f};
    RowDot<25>::run(hv2, w01, w23, a01e, a01o, a23e, a23o);
    float p[4] = {a01e.x + a01o.x, a01e.y + a01o.y, a23e.x + a23o.x, a23e.y + a23o.y};
#pragma unroll
    for (int j = 0; j < 4; ++j) p[j] += xor16(p[j]);
#pragma unroll
    for (int j = 0; j < 4; ++j) p[j] += xor32(p[j]);
    const float ig = sigm(bh4[0] + p[0]), fg = sigm(bh4[1] + p[1]);
    const float cg = ftanh(bh4[2] + p[2]), og = sigm(bh4[3] + p[3]);
    const float c = fg * creg + ig * cg;
    const float h = og * ftanh(c);
    creg = c;
    if (act && q == 0) hn[hw] = h;
    ph = h; pc = c;
    pav = q == 0 ? ig : q == 1 ? fg : q == 2 ? cg : og;
    __syncthreads();
  }
  if (a.S > 0 && act) {
    if (q == 0) { hb[0] = ph; cb[0] = pc; }
    gp[0] = pav;
  }
}

// ------------------------------------------------------------------ F3 / F4
// F1 (448 threads) with every lane finishing all four gates itself (after the
// two quad DPP adds every lane of the quad holds all four sums): four
// independent activations instead of one activation followed by four quad
// broadcasts on the step's dependent chain; the x part of all four gates as
// one float4 LDS read.  F4: K split in contiguous quarters of 25 (h image
// padded to 28 per quarter) so only real k are multiplied (12 pairs + 1).
template <bool EXACT>
__global__ void __launch_bounds__(448) f3_kernel(Args a) {
  constexpr int KQ = 28, NTH = 448;
  __shared__ __attribute__((aligned(16))) float hS[2][4 * KQ];
  extern __shared__ __attribute__((aligned(16))) float4 xP4[];     // [S][112] (i, f, g, o)
  const int B = a.B, b = blockIdx.x;
  const int tid = threadIdx.x, u = tid >> 2, q = tid & 3;
  const bool act = u < H;
  const int uc = act ? u : H - 1;
  const int g = q * H + uc;
  const int64_t BH = (int64_t)B * H;
  for (int e = tid; e < a.S * 112; e += NTH) {
    const int un = e % 112 < H ? e % 112 : H - 1;
    xP4[e] = float4{a.b_hh[un] + a.b_ih[un], a.b_hh[H + un] + a.b_ih[H + un],
                    a.b_hh[2 * H + un] + a.b_ih[2 * H + un], a.b_hh[3 * H + un] + a.b_ih[3 * H + un]};
  }
  float creg = a.c0[(int64_t)b * H + uc];
  if (act && q == 0) a.cbuf[(int64_t)b * H + u] = creg;
  auto pos = [](int k) { return EXACT ? (k / 25) * KQ + k % 25 : k; };
  for (int e = tid; e < 4 * KQ; e += NTH) { hS[0][e] = 0.f; hS[1][e] = 0.f; }
  __syncthreads();
  for (int e = tid; e < H; e += NTH) {
    const float v = a.h0[(int64_t)b * H + e];
    hS[0][pos(e)] = v;
    a.hbuf[(int64_t)b * H + e] = v;
  }
  vf2 wv[4][KQ / 2];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float* r = a.w_hh + (int64_t)(j * H + uc) * H;
#pragma unroll
    for (int i = 0; i < KQ / 2; ++i) {
      if (EXACT) {
        const int k0 = 25 * q + 2 * i;
        wv[j][i] = vf2{2 * i < 25 ? r[k0] : 0.f, 2 * i + 1 < 25 ? r[k0 + 1] : 0.f};
      } else {
        const int k = 16 * (i >> 1) + 4 * q + 2 * (i & 1);
        wv[j][i] = vf2{k < H ? r[k] : 0.f, k + 1 < H ? r[k + 1] : 0.f};
      }
    }
  }
  __syncthreads();
  float* hb = a.hbuf + BH + (int64_t)b * H + uc;
  float* cb = a.cbuf + BH + (int64_t)b * H + uc;
  float* gp = a.gates + (int64_t)b * G4 + g;
  const int64_t gstep = (int64_t)B * G4;
  const int hw = pos(uc);
  float ph = 0.f, pc = 0.f, pav = 0.f;
  for (int t = 0; t < a.S; ++t) {
    const float* hp = hS[t & 1] + (EXACT ? KQ * q : 4 * q);
    float* hn = hS[(t + 1) & 1];
    float2 hv[KQ / 2];
    const float4* h4 = reinterpret_cast<const float4*>(hp);
#pragma unroll
    for (int i = 0; i < KQ / 4; ++i) {
      const float4 v = h4[EXACT ? i : 4 * i];
      hv[2 * i] = float2{v.x, v.y};
      hv[2 * i + 1] = float2{v.z, v.w};
    }
    const float4 x4 = xP4[t * 112 + u];
    if (t > 0 && act) {
      if (q == 0) {
        hb[0] = ph; hb += BH;
        cb[0] = pc; cb += BH;
      }
      gp[0] = pav; gp += gstep;
    }
    float pj[4];
    if (EXACT) {
      vf2 pp[4] = {vf2{0.f, 0.f}, vf2{0.f, 0.f}, vf2{0.f, 0.f}, vf2{0.f, 0.f}};
#pragma unroll
      for (int i = 0; i < 12; ++i) {
        const vf2 h2v = vf2{hv[i].x, hv[i].y};
#pragma unroll
        for (int j = 0; j < 4; ++j) pp[j] = __builtin_elementwise_fma(h2v, wv[j][i], pp[j]);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) pj[j] = fmaf(hv[12].x, wv[j][12].x, pp[j].x + pp[j].y);
    } else {
      vf2 pp[4] = {vf2{0.f, 0.f}, vf2{0.f, 0.f}, vf2{0.f, 0.f}, vf2{0.f, 0.f}};
#pragma unroll
      for (int i = 0; i < KQ / 2; ++i) {
        const vf2 h2v = vf2{hv[i].x, hv[i].y};
#pragma unroll
        for (int j = 0; j < 4; ++j) pp[j] = __builtin_elementwise_fma(h2v, wv[j][i], pp[j]);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) pj[j] = pp[j].x + pp[j].y;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      pj[j] += dpp_x1(pj[j]);
      pj[j] += dpp_x2(pj[j]);
    }
    const float ig = sigm(x4.x + pj[0]), fg = sigm(x4.y + pj[1]);
    const float cg = ftanh(x4.z + pj[2]), og = sigm(x4.w + pj[3]);
    const float c = fg * creg + ig * cg;
    const float h = og * ftanh(c);
    creg = c;
    if (act && q == 0) hn[hw] = h;
    ph = h; pc = c;
    pav = q == 0 ? ig : q == 1 ? fg : q == 2 ? cg : og;
    __syncthreads();
  }
  if (a.S > 0 && act) {
    if (q == 0) { hb[0] = ph; cb[0] = pc; }
    gp[0] = pav;
  }
}

// ------------------------------------------------------------------ BPTT
struct BArgs {
  const float* dh; const float* gates; const float* cbuf; const float* w_hh;
  int S, B;
  float* dgates;
};
__device__ __forceinline__ float dpp_hmirror(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x141, 0xF, 0xF, false));
}
__device__ __forceinline__ float dpp_ror8(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x128, 0xF, 0xF, false));
}
// B0: the product body (lstm_bwd_q_body<25>); CH = 2 (product) or 4 FMA
// chains per lane (even / odd rows); NTH 512 (product) or 448
template <int CH, int NTH>
__global__ void __launch_bounds__(512) b_kernel(BArgs a) {
  constexpr int BR = 25, BRP = 28;
  __shared__ __attribute__((aligned(16))) float dG[2][16 * BRP];
  const int B = a.B, b = blockIdx.x;
  const int tid = threadIdx.x, u = tid >> 2, q = tid & 3;
  const bool act = u < H;
  const int uc = act ? u : H - 1;
  const int g = q * H + uc;
  const int64_t BH = (int64_t)B * H;
  const int ug = tid >> 4, rr = tid & 15;
  for (int e = tid; e < 2 * 16 * BRP; e += NTH) (&dG[0][0])[e] = 0.f;
  vf2 w01[BR], w23[BR];
  {
    const bool ok = 4 * ug + 3 < H;
#pragma unroll
    for (int i = 0; i < BR; ++i) {
      const int r = rr * BR + i;
      const float* row = a.w_hh + (int64_t)r * H;
      const float4 v = ok ? *reinterpret_cast<const float4*>(row + 4 * ug) : float4{0.f, 0.f, 0.f, 0.f};
      w01[i] = vf2{v.x, v.y};
      w23[i] = vf2{v.z, v.w};
    }
  }
  const int dgi = (g / BR) * BRP + g % BR;
  float gq, ct, ctm, dho, gqn, ctn, ctmn, dhon;
  auto fetch = [&](int t, float& G_, float& C, float& CM, float& DH) {
    G_ = a.gates[((int64_t)t * B + b) * G4 + g];
    C = a.cbuf[(int64_t)(t + 1) * BH + (int64_t)b * H + uc];
    CM = a.cbuf[(int64_t)t * BH + (int64_t)b * H + uc];
    DH = a.dh[(int64_t)t * BH + (int64_t)b * H + uc];
  };
  fetch(a.S - 1, gq, ct, ctm, dho);
  fetch(a.S >= 2 ? a.S - 2 : 0, gqn, ctn, ctmn, dhon);
  float dcreg = 0.f, dhr = 0.f;
  __syncthreads();
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
    float pu[4];
    if (CH == 2) {
      vf2 p01 = {0.f, 0.f}, p23 = {0.f, 0.f};
#pragma unroll
      for (int i = 0; i < BR; ++i) {
        const float d = (i & 3) == 0 ? dv[i >> 2].x : (i & 3) == 1 ? dv[i >> 2].y
                      : (i & 3) == 2 ? dv[i >> 2].z : dv[i >> 2].w;
        p01 = __builtin_elementwise_fma(vf2{d, d}, w01[i], p01);
        p23 = __builtin_elementwise_fma(vf2{d, d}, w23[i], p23);
      }
      pu[0] = p01.x; pu[1] = p01.y; pu[2] = p23.x; pu[3] = p23.y;
    } else {
      vf2 p01e = {0.f, 0.f}, p23e = {0.f, 0.f}, p01o = {0.f, 0.f}, p23o = {0.f, 0.f};
#pragma unroll
      for (int i = 0; i < BR; ++i) {
        const float d = (i & 3) == 0 ? dv[i >> 2].x : (i & 3) == 1 ? dv[i >> 2].y
                      : (i & 3) == 2 ? dv[i >> 2].z : dv[i >> 2].w;
        if (i & 1) {
          p01o = __builtin_elementwise_fma(vf2{d, d}, w01[i], p01o);
          p23o = __builtin_elementwise_fma(vf2{d, d}, w23[i], p23o);
        } else {
          p01e = __builtin_elementwise_fma(vf2{d, d}, w01[i], p01e);
          p23e = __builtin_elementwise_fma(vf2{d, d}, w23[i], p23e);
        }
      }
      const vf2 p01 = p01e + p01o, p23 = p23e + p23o;
      pu[0] = p01.x; pu[1] = p01.y; pu[2] = p23.x; pu[3] = p23.y;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      pu[k] += dpp_x1(pu[k]);
      pu[k] += dpp_x2(pu[k]);
      pu[k] += dpp_hmirror(pu[k]);
      pu[k] += dpp_ror8(pu[k]);
    }
    const int k = u & 3;
    dhr = k == 0 ? pu[0] : k == 1 ? pu[1] : k == 2 ? pu[2] : pu[3];
  }
}
typedef void (*BFn)(BArgs);
static float runb(BFn k, const BArgs& a, int iters, int nt) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<float> ts;
  for (int it = 0; it < iters + 3; ++it) {
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(k, dim3(a.B), dim3(nt), 0, 0, a);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (it >= 3) ts.push_back(ms * 1e3f);
  }
  std::sort(ts.begin(), ts.end());
  return ts[ts.size() / 2];
}

typedef void (*KFn)(Args);
static float run(KFn k, const Args& a, int iters, int nt, size_t lds = 0) {
  if (lds > 64 * 1024)
    CK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<float> ts;
  for (int it = 0; it < iters + 3; ++it) {
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(k, dim3(a.B), dim3(nt), lds, 0, a);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (it >= 3) ts.push_back(ms * 1e3f);
  }
  std::sort(ts.begin(), ts.end());
  return ts[ts.size() / 2];
}

int main() {
  const int B = 128, SMAX = 41;
  std::vector<float> hwhh((size_t)G4 * H), hbih(G4), hbhh(G4), hh0((size_t)B * H), hc0((size_t)B * H);
  srand(1);
  auto rnd = [] { return (float)rand() / RAND_MAX * 2.f - 1.f; };
  for (auto& v : hwhh) v = 0.2f * rnd();
  for (auto& v : hbih) v = 0.3f * rnd();
  for (auto& v : hbhh) v = 0.3f * rnd();
  for (auto& v : hh0) v = 0.5f * rnd();
  for (auto& v : hc0) v = 0.5f * rnd();
  auto up = [](const std::vector<float>& h) {
    float* d;
    CK(hipMalloc(&d, h.size() * 4));
    CK(hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    return d;
  };
  float *dwhh = up(hwhh), *dbih = up(hbih), *dbhh = up(hbhh), *dh0 = up(hh0), *dc0 = up(hc0);
  const int NV = 7;
  float *hb[NV], *cb[NV], *gt[NV];
  for (int v = 0; v < NV; ++v) {
    CK(hipMalloc(&hb[v], (size_t)(SMAX + 1) * B * H * 4));
    CK(hipMalloc(&cb[v], (size_t)(SMAX + 1) * B * H * 4));
    CK(hipMalloc(&gt[v], (size_t)SMAX * B * G4 * 4));
  }
  KFn ks[NV] = {f0_kernel<512, 0>, f0_kernel<448, 0>, f2_kernel, f0_kernel<512, 1>, f0_kernel<512, 2>,
                f3_kernel<false>, f3_kernel<true>};
  const int nts[NV] = {512, 448, 448, 512, 512, 448, 448};
  const char* names[NV] = {"F0", "F1", "F2", "F0n_noFMA", "F0l_noLDS", "F3", "F4"};
  const int Ss[3] = {1, 21, 41};
  for (int v = 0; v < NV; ++v) {
    float t[3];
    for (int si = 0; si < 3; ++si) {
      Args a{dwhh, dbih, dbhh, dh0, dc0, Ss[si], B, hb[v], cb[v], gt[v]};
      t[si] = run(ks[v], a, 30, nts[v], v >= 5 ? (size_t)Ss[si] * 112 * 16 : 0);
    }
    printf("{\"variant\": \"%s\", \"us_S1\": %.2f, \"us_S21\": %.2f, \"us_S41\": %.2f, \"us_per_step\": %.4f}\n",
           names[v], t[0], t[1], t[2], (t[2] - t[0]) / 40.f);
    fflush(stdout);
  }
  auto dl = [](const float* d, size_t n) {
    std::vector<float> h(n);
    CK(hipMemcpy(h.data(), d, n * 4, hipMemcpyDeviceToHost));
    return h;
  };
  const size_t nh = (size_t)(SMAX + 1) * B * H, ng = (size_t)SMAX * B * G4;
  auto h0v = dl(hb[0], nh), c0v = dl(cb[0], nh), g0v = dl(gt[0], ng);
  for (int v : {1, 2, 5, 6}) {
    auto h1v = dl(hb[v], nh), c1v = dl(cb[v], nh), g1v = dl(gt[v], ng);
    double dh = 0, dc = 0, dg = 0, mh = 0;
    for (size_t i = 0; i < nh; ++i) {
      dh = std::max(dh, (double)fabsf(h0v[i] - h1v[i]));
      dc = std::max(dc, (double)fabsf(c0v[i] - c1v[i]));
      mh = std::max(mh, (double)fabsf(h0v[i]));
    }
    for (size_t i = 0; i < ng; ++i) dg = std::max(dg, (double)fabsf(g0v[i] - g1v[i]));
    printf("{\"check\": \"%s vs F0 at S=41\", \"max_dh\": %.3g, \"max_dc\": %.3g, \"max_dgates\": %.3g, \"max_h\": %.3g}\n",
           names[v], dh, dc, dg, mh);
  }
  {   // BPTT variants at S = 1 / 21 / 41 over F0's gates / cbuf and random dh
    std::vector<float> hdh((size_t)SMAX * B * H);
    for (auto& v : hdh) v = 0.1f * rnd();
    float* ddh = up(hdh);
    const int NB = 3;
    float* dg[NB];
    for (int i = 0; i < NB; ++i) CK(hipMalloc(&dg[i], (size_t)SMAX * B * G4 * 4));
    BFn bk[NB] = {b_kernel<2, 512>, b_kernel<4, 512>, b_kernel<4, 448>};
    const int bn[NB] = {512, 512, 448};
    const char* bnames[NB] = {"B0", "B1_4chains", "B2_4chains_448"};
    for (int v = 0; v < NB; ++v) {
      float t[3];
      for (int si = 0; si < 3; ++si) {
        BArgs ba{ddh, gt[0], cb[0], dwhh, Ss[si], B, dg[v]};
        t[si] = runb(bk[v], ba, 30, bn[v]);
      }
      printf("{\"variant\": \"%s\", \"us_S1\": %.2f, \"us_S21\": %.2f, \"us_S41\": %.2f, \"us_per_step\": %.4f}\n",
             bnames[v], t[0], t[1], t[2], (t[2] - t[0]) / 40.f);
      fflush(stdout);
    }
    // each variant's last run was at S = 41
    auto d0 = dl(dg[0], ng);
    for (int v = 1; v < NB; ++v) {
      auto d1 = dl(dg[v], ng);
      double md = 0, mx = 0;
      for (size_t i = 0; i < ng; ++i) {
        md = std::max(md, (double)fabsf(d0[i] - d1[i]));
        mx = std::max(mx, (double)fabsf(d0[i]));
      }
      printf("{\"check\": \"%s vs B0 at S=41\", \"max_ddgates\": %.3g, \"max_dgates\": %.3g}\n", bnames[v], md, mx);
    }
  }
  return 0;
}
