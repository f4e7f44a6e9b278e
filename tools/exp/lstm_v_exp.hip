// LSTM VALU recurrence experiments at a rank's batch (diagnostic only, not
// product code): 128 segments, H 100, x width 42 (fused input projection),
// one segment per workgroup.  Times each variant at S = 1 / 21 / 41 steps
// (median of 30 launches, HIP events) -> prologue and per-step cost, and
// checks every variant's hbuf / cbuf / gates against V0 (max abs diff).
//   V0  the product kernel's form (lstm_fwd_v_kernel<1, 104, 48>): thread
//       (u, q) owns gate column q*H + u with its whole W_hh row; every thread
//       reads all of h_{t-1} from LDS each step (26 x ds_read_b128 per wave)
//   V1  K split over the quad: thread (u, q) owns the four gate rows of unit u
//       over k in [q*KQ, (q+1)*KQ): a step reads KQ h values, the four
//       partial sums meet through two quad DPP adds each; the x part is
//       precomputed the same way (K split of W_ih)
//   hipcc -O3 --offload-arch=gfx950 -fno-slp-vectorize tools/exp/lstm_v_exp.hip -o /tmp/lstm_v_exp
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int H = 100, G4 = 400, DIN = 42, KP = 104, KX = 48, NT = 448;

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
// v + lane (l ^ 1) / (l ^ 2) of the quad
__device__ __forceinline__ float qx1(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false));  // [1,0,3,2]
}
__device__ __forceinline__ float qx2(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, false));  // [2,3,0,1]
}

typedef float vf2 __attribute__((ext_vector_type(2)));

struct Args {
  const float* x; int ldx; const float* w_ih; const float* b_ih; const float* w_hh;
  const float* b_hh; const float* h0; const float* c0; int S, B;
  float* hbuf; float* cbuf; float* gates;
};

// ---------------------------------------------------------------- V0
constexpr int kVC = 4;
__device__ __forceinline__ void v_dot_pipelined(const float4* __restrict__ v, const float (&w)[KP],
                                                float& s0, float& s1, float& s2, float& s3) {
  constexpr int N4 = KP / 4, NC = (N4 + kVC - 1) / kVC;
  float4 buf[2][kVC];
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
        s0 = fmaf(hv.x, w[4 * k4], s0);
        s1 = fmaf(hv.y, w[4 * k4 + 1], s1);
        s2 = fmaf(hv.z, w[4 * k4 + 2], s2);
        s3 = fmaf(hv.w, w[4 * k4 + 3], s3);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

__global__ void __launch_bounds__(NT) v0_kernel(Args a) {
  __shared__ __attribute__((aligned(16))) float hS[2][KP];
  extern __shared__ __attribute__((aligned(16))) float xS[];
  float* xP = xS + ((a.S * KX + 3) & ~3);
  const int B = a.B;
  const int tid = threadIdx.x, u = tid >> 2, q = tid & 3;
  const bool act = u < H;
  const int uc = act ? u : H - 1;
  const int g = q * H + uc;
  const int b = blockIdx.x;
  const int64_t BH = (int64_t)B * H;
  float w[KP];
#pragma unroll
  for (int k = 0; k < KP; ++k) {
    const float x = a.w_hh[(int64_t)g * H + (k < H ? k : H - 1)];
    w[k] = k < H ? x : 0.f;
  }
  float bh = a.b_hh[g] + a.b_ih[g];
  float wx[KX];
#pragma unroll
  for (int k = 0; k < KX; ++k) {
    const float x = a.w_ih[(int64_t)g * DIN + (k < DIN ? k : DIN - 1)];
    wx[k] = k < DIN ? x : 0.f;
  }
  for (int e = tid; e < a.S * KX; e += NT) {
    const int t = e / KX, k = e - t * KX;
    xS[e] = k < DIN ? a.x[((int64_t)t * B + b) * a.ldx + k] : 0.f;
  }
  float creg = a.c0[(int64_t)b * H + uc];
  if (act && q == 0) a.cbuf[(int64_t)b * H + u] = creg;
  for (int e = tid; e < KP; e += NT) {
    const float v = e < H ? a.h0[(int64_t)b * H + e] : 0.f;
    hS[0][e] = v;
    hS[1][e] = 0.f;
    if (e < H) a.hbuf[(int64_t)b * H + e] = v;
  }
  __syncthreads();
  for (int t = 0; t < a.S; ++t) {
    const float4* xp = reinterpret_cast<const float4*>(xS + t * KX);
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
    xP[t * NT + tid] = (s0 + s1) + (s2 + s3);
  }
  __builtin_amdgcn_s_waitcnt(0x0F70);
  for (int t = 0; t < a.S; ++t) {
    const float* hp = hS[t & 1];
    float* hn = hS[(t + 1) & 1];
    const float xacc = xP[t * NT + tid];
    float acc0 = 0.f, acc1 = 0.f, acc2 = 0.f, acc3 = 0.f;
    v_dot_pipelined(reinterpret_cast<const float4*>(hp), w, acc0, acc1, acc2, acc3);
    const float pre = xacc + (((acc0 + acc1) + (acc2 + acc3)) + bh);
    const float av = q == 2 ? ftanh(pre) : sigm(pre);
    const float ig = quad_bcast<0>(av), fg = quad_bcast<1>(av);
    const float cg = quad_bcast<2>(av), og = quad_bcast<3>(av);
    const float c = fg * creg + ig * cg;
    const float h = og * ftanh(c);
    creg = c;
    if (act) {
      if (q == 0) {
        hn[u] = h;
        a.hbuf[(int64_t)(t + 1) * BH + (int64_t)b * H + u] = h;
        a.cbuf[(int64_t)(t + 1) * BH + (int64_t)b * H + u] = c;
      }
      a.gates[((int64_t)t * B + b) * G4 + g] = av;
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------- V1
constexpr int KQ = KP / 4;     // 26 h values per lane
constexpr int XQ = KX / 4;     // 12 x values per lane
__global__ void __launch_bounds__(NT) v1_kernel(Args a) {
  __shared__ __attribute__((aligned(16))) float hS[2][KP];
  extern __shared__ __attribute__((aligned(16))) float xS[];
  float* xP = xS + ((a.S * KX + 3) & ~3);          // [S][NT]: x part of gate column q*H+u at tid
  const int B = a.B;
  const int tid = threadIdx.x, u = tid >> 2, q = tid & 3;
  const bool act = u < H;
  const int uc = act ? u : H - 1;
  const int b = blockIdx.x;
  const int64_t BH = (int64_t)B * H;
  // W_hh rows j*H + u (j = gate), k in [q*KQ, q*KQ + KQ)
  float w[4][KQ];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int kk = 0; kk < KQ; ++kk) {
      const int k = q * KQ + kk;
      const float x = a.w_hh[(int64_t)(j * H + uc) * H + (k < H ? k : H - 1)];
      w[j][kk] = k < H ? x : 0.f;
    }
  const int g = q * H + uc;                        // the gate column this lane finishes
  const float bh = a.b_hh[g] + a.b_ih[g];
  for (int e = tid; e < a.S * KX; e += NT) {
    const int t = e / KX, k = e - t * KX;
    xS[e] = k < DIN ? a.x[((int64_t)t * B + b) * a.ldx + k] : 0.f;
  }
  float creg = a.c0[(int64_t)b * H + uc];
  if (act && q == 0) a.cbuf[(int64_t)b * H + u] = creg;
  for (int e = tid; e < KP; e += NT) {
    const float v = e < H ? a.h0[(int64_t)b * H + e] : 0.f;
    hS[0][e] = v;
    hS[1][e] = 0.f;
    if (e < H) a.hbuf[(int64_t)b * H + e] = v;
  }
  __syncthreads();
  // x parts: W_ih rows j*H + u over x columns [q*XQ, q*XQ + XQ), quad sum
  {
    float wx[4][XQ];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int kk = 0; kk < XQ; ++kk) {
        const int k = q * XQ + kk;
        const float x = a.w_ih[(int64_t)(j * H + uc) * DIN + (k < DIN ? k : DIN - 1)];
        wx[j][kk] = k < DIN ? x : 0.f;
      }
    for (int t = 0; t < a.S; ++t) {
      const float4* xp = reinterpret_cast<const float4*>(xS + t * KX + q * XQ);
      float p[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int k4 = 0; k4 < XQ / 4; ++k4) {
        const float4 v = xp[k4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          p[j] = fmaf(v.x, wx[j][4 * k4], p[j]);
          p[j] = fmaf(v.y, wx[j][4 * k4 + 1], p[j]);
          p[j] = fmaf(v.z, wx[j][4 * k4 + 2], p[j]);
          p[j] = fmaf(v.w, wx[j][4 * k4 + 3], p[j]);
        }
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        p[j] += qx1(p[j]);
        p[j] += qx2(p[j]);
      }
      const float mine = q == 0 ? p[0] : q == 1 ? p[1] : q == 2 ? p[2] : p[3];
      xP[t * NT + tid] = mine + bh;
    }
  }
  __builtin_amdgcn_s_waitcnt(0x0F70);
  for (int t = 0; t < a.S; ++t) {
    const float* hp = hS[t & 1] + q * KQ;
    float* hn = hS[(t + 1) & 1];
    const float xacc = xP[t * NT + tid];
    float p[4] = {0.f, 0.f, 0.f, 0.f};
    // 26 h values: 13 ds_read_b64 (q*KQ*4 bytes is 8-byte aligned)
    const float2* h2 = reinterpret_cast<const float2*>(hp);
    float2 hv[KQ / 2];
#pragma unroll
    for (int i = 0; i < KQ / 2; ++i) hv[i] = h2[i];
#pragma unroll
    for (int i = 0; i < KQ / 2; ++i) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        p[j] = fmaf(hv[i].x, w[j][2 * i], p[j]);
        p[j] = fmaf(hv[i].y, w[j][2 * i + 1], p[j]);
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      p[j] += qx1(p[j]);
      p[j] += qx2(p[j]);
    }
    const float mine = q == 0 ? p[0] : q == 1 ? p[1] : q == 2 ? p[2] : p[3];
    const float pre = xacc + mine;
    const float av = q == 2 ? ftanh(pre) : sigm(pre);
    const float ig = quad_bcast<0>(av), fg = quad_bcast<1>(av);
    const float cg = quad_bcast<2>(av), og = quad_bcast<3>(av);
    const float c = fg * creg + ig * cg;
    const float h = og * ftanh(c);
    creg = c;
    if (act) {
      if (q == 0) {
        hn[u] = h;
        a.hbuf[(int64_t)(t + 1) * BH + (int64_t)b * H + u] = h;
        a.cbuf[(int64_t)(t + 1) * BH + (int64_t)b * H + u] = c;
      }
      a.gates[((int64_t)t * B + b) * G4 + g] = av;
    }
    __syncthreads();
  }
}


// ---------------------------------------------------------------- V0 + ticks
// per wave (lane 0): accumulated shader cycles (s_memtime) of each phase:
// [0] prologue W loads, [1] x staging + h0 + sync, [2] x parts, [3] step: x
// read + dot, [4] step: activation + quad exchange + cell, [5] step: stores,
// [6] step: barrier
__device__ unsigned long long g_ticks[8][8];
__global__ void __launch_bounds__(NT) v0t_kernel(Args a) {
  __shared__ __attribute__((aligned(16))) float hS[2][KP];
  extern __shared__ __attribute__((aligned(16))) float xS[];
  float* xP = xS + ((a.S * KX + 3) & ~3);
  const int B = a.B;
  const int tid = threadIdx.x, u = tid >> 2, q = tid & 3;
  const bool act = u < H;
  const int uc = act ? u : H - 1;
  const int g = q * H + uc;
  const int b = blockIdx.x;
  const int64_t BH = (int64_t)B * H;
  unsigned long long tk[7] = {0, 0, 0, 0, 0, 0, 0};
  unsigned long long tp = __builtin_amdgcn_s_memtime();
  auto tick = [&](int i) {
    const unsigned long long n = __builtin_amdgcn_s_memtime();
    tk[i] += n - tp;
    tp = n;
  };
  float w[KP];
#pragma unroll
  for (int k = 0; k < KP; ++k) {
    const float x = a.w_hh[(int64_t)g * H + (k < H ? k : H - 1)];
    w[k] = k < H ? x : 0.f;
  }
  float bh = a.b_hh[g] + a.b_ih[g];
  float wx[KX];
#pragma unroll
  for (int k = 0; k < KX; ++k) {
    const float x = a.w_ih[(int64_t)g * DIN + (k < DIN ? k : DIN - 1)];
    wx[k] = k < DIN ? x : 0.f;
  }
  __builtin_amdgcn_s_waitcnt(0x0F70);
  tick(0);
  for (int e = tid; e < a.S * KX; e += NT) {
    const int t = e / KX, k = e - t * KX;
    xS[e] = k < DIN ? a.x[((int64_t)t * B + b) * a.ldx + k] : 0.f;
  }
  float creg = a.c0[(int64_t)b * H + uc];
  if (act && q == 0) a.cbuf[(int64_t)b * H + u] = creg;
  for (int e = tid; e < KP; e += NT) {
    const float v = e < H ? a.h0[(int64_t)b * H + e] : 0.f;
    hS[0][e] = v;
    hS[1][e] = 0.f;
    if (e < H) a.hbuf[(int64_t)b * H + e] = v;
  }
  __syncthreads();
  tick(1);
  for (int t = 0; t < a.S; ++t) {
    const float4* xp = reinterpret_cast<const float4*>(xS + t * KX);
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
    xP[t * NT + tid] = (s0 + s1) + (s2 + s3);
  }
  __builtin_amdgcn_s_waitcnt(0x0F70);
  __builtin_amdgcn_s_waitcnt(0xC07F);
  tick(2);
  for (int t = 0; t < a.S; ++t) {
    const float* hp = hS[t & 1];
    float* hn = hS[(t + 1) & 1];
    const float xacc = xP[t * NT + tid];
    float acc0 = 0.f, acc1 = 0.f, acc2 = 0.f, acc3 = 0.f;
    v_dot_pipelined(reinterpret_cast<const float4*>(hp), w, acc0, acc1, acc2, acc3);
    const float pre = xacc + (((acc0 + acc1) + (acc2 + acc3)) + bh);
    __builtin_amdgcn_sched_barrier(0);
    tick(3);
    const float av = q == 2 ? ftanh(pre) : sigm(pre);
    const float ig = quad_bcast<0>(av), fg = quad_bcast<1>(av);
    const float cg = quad_bcast<2>(av), og = quad_bcast<3>(av);
    const float c = fg * creg + ig * cg;
    const float h = og * ftanh(c);
    creg = c;
    __builtin_amdgcn_sched_barrier(0);
    tick(4);
    if (act) {
      if (q == 0) {
        hn[u] = h;
        a.hbuf[(int64_t)(t + 1) * BH + (int64_t)b * H + u] = h;
        a.cbuf[(int64_t)(t + 1) * BH + (int64_t)b * H + u] = c;
      }
      a.gates[((int64_t)t * B + b) * G4 + g] = av;
    }
    __builtin_amdgcn_sched_barrier(0);
    tick(5);
    __syncthreads();
    tick(6);
  }
  if (b == 0 && (tid & 63) == 0) {
    for (int i = 0; i < 7; ++i) g_ticks[tid >> 6][i] = tk[i];
  }
}

// V0 with the prologue's weight rows loaded as 16-byte (W_hh) / 8-byte (W_ih)
// vectors instead of one float per load
__global__ void __launch_bounds__(NT) v0v_kernel(Args a) {
  __shared__ __attribute__((aligned(16))) float hS[2][KP];
  extern __shared__ __attribute__((aligned(16))) float xS[];
  float* xP = xS + ((a.S * KX + 3) & ~3);
  const int B = a.B;
  const int tid = threadIdx.x, u = tid >> 2, q = tid & 3;
  const bool act = u < H;
  const int uc = act ? u : H - 1;
  const int g = q * H + uc;
  const int b = blockIdx.x;
  const int64_t BH = (int64_t)B * H;
  float w[KP];
  {
    const float4* r4 = reinterpret_cast<const float4*>(a.w_hh + (int64_t)g * H);
#pragma unroll
    for (int k4 = 0; k4 < H / 4; ++k4) {
      const float4 v = r4[k4];
      w[4 * k4] = v.x; w[4 * k4 + 1] = v.y; w[4 * k4 + 2] = v.z; w[4 * k4 + 3] = v.w;
    }
#pragma unroll
    for (int k = H; k < KP; ++k) w[k] = 0.f;
  }
  float bh = a.b_hh[g] + a.b_ih[g];
  float wx[KX];
  {
    const float2* r2 = reinterpret_cast<const float2*>(a.w_ih + (int64_t)g * DIN);
#pragma unroll
    for (int k2 = 0; k2 < DIN / 2; ++k2) {
      const float2 v = r2[k2];
      wx[2 * k2] = v.x; wx[2 * k2 + 1] = v.y;
    }
#pragma unroll
    for (int k = DIN; k < KX; ++k) wx[k] = 0.f;
  }
  for (int e = tid; e < a.S * KX; e += NT) {
    const int t = e / KX, k = e - t * KX;
    xS[e] = k < DIN ? a.x[((int64_t)t * B + b) * a.ldx + k] : 0.f;
  }
  float creg = a.c0[(int64_t)b * H + uc];
  if (act && q == 0) a.cbuf[(int64_t)b * H + u] = creg;
  for (int e = tid; e < KP; e += NT) {
    const float v = e < H ? a.h0[(int64_t)b * H + e] : 0.f;
    hS[0][e] = v;
    hS[1][e] = 0.f;
    if (e < H) a.hbuf[(int64_t)b * H + e] = v;
  }
  __syncthreads();
  for (int t = 0; t < a.S; ++t) {
    const float4* xp = reinterpret_cast<const float4*>(xS + t * KX);
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
    xP[t * NT + tid] = (s0 + s1) + (s2 + s3);
  }
  __builtin_amdgcn_s_waitcnt(0x0F70);
  for (int t = 0; t < a.S; ++t) {
    const float* hp = hS[t & 1];
    float* hn = hS[(t + 1) & 1];
    const float xacc = xP[t * NT + tid];
    float acc0 = 0.f, acc1 = 0.f, acc2 = 0.f, acc3 = 0.f;
    v_dot_pipelined(reinterpret_cast<const float4*>(hp), w, acc0, acc1, acc2, acc3);
    const float pre = xacc + (((acc0 + acc1) + (acc2 + acc3)) + bh);
    const float av = q == 2 ? ftanh(pre) : sigm(pre);
    const float ig = quad_bcast<0>(av), fg = quad_bcast<1>(av);
    const float cg = quad_bcast<2>(av), og = quad_bcast<3>(av);
    const float c = fg * creg + ig * cg;
    const float h = og * ftanh(c);
    creg = c;
    if (act) {
      if (q == 0) {
        hn[u] = h;
        a.hbuf[(int64_t)(t + 1) * BH + (int64_t)b * H + u] = h;
        a.cbuf[(int64_t)(t + 1) * BH + (int64_t)b * H + u] = c;
      }
      a.gates[((int64_t)t * B + b) * G4 + g] = av;
    }
    __syncthreads();
  }
}

__global__ void empty_kernel(Args a) {
  if (a.S < 0) a.hbuf[threadIdx.x] = 0.f;
}

// ---------------------------------------------------------------- V2
// V1's K-split, plus: vector weight loads (float2 runs of each lane's k range),
// W_hh loads issued before the x-part loop (in flight while it runs), per-step
// pointers advanced instead of recomputed, and the step's global stores
// (hbuf, cbuf, gates) issued AFTER the barrier, where they overlap the next
// step's LDS reads instead of delaying the barrier.  TICKS: per-wave phase
// cycles into g_ticks2.
__device__ unsigned long long g_ticks2[8][8];
template <bool TICKS>
__global__ void __launch_bounds__(NT) v2_kernel(Args a) {
  __shared__ __attribute__((aligned(16))) float hS[2][KP];
  extern __shared__ __attribute__((aligned(16))) float xS[];
  float* xP = xS + ((a.S * KX + 3) & ~3);
  const int B = a.B;
  const int tid = threadIdx.x, u = tid >> 2, q = tid & 3;
  const bool act = u < H;
  const int uc = act ? u : H - 1;
  const int b = blockIdx.x;
  const int64_t BH = (int64_t)B * H;
  unsigned long long tk[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long tp = TICKS ? __builtin_amdgcn_s_memtime() : 0;
  auto tick = [&](int i) {
    if (TICKS) {
      const unsigned long long n = __builtin_amdgcn_s_memtime();
      tk[i] += n - tp;
      tp = n;
    }
  };
  const int g = q * H + uc;
  // W_ih rows j*H + u over x columns [q*XQ, q*XQ + XQ): float2 runs (row
  // stride 168 B, q*XQ*4 = 48q: 8-byte aligned); columns >= DIN read as 0
  float wx[4][XQ];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float* r = a.w_ih + (int64_t)(j * H + uc) * DIN;
#pragma unroll
    for (int kk = 0; kk < XQ; kk += 2) {
      const int k = q * XQ + kk;
      float2 v = k + 1 < DIN ? *reinterpret_cast<const float2*>(r + k) : float2{0.f, 0.f};
      wx[j][kk] = v.x;
      wx[j][kk + 1] = v.y;
    }
  }
  const float bh = a.b_hh[g] + a.b_ih[g];
  for (int e = tid; e < a.S * KX; e += NT) {
    const int t = e / KX, k = e - t * KX;
    xS[e] = k < DIN ? a.x[((int64_t)t * B + b) * a.ldx + k] : 0.f;
  }
  float creg = a.c0[(int64_t)b * H + uc];
  if (act && q == 0) a.cbuf[(int64_t)b * H + u] = creg;
  for (int e = tid; e < KP; e += NT) {
    const float v = e < H ? a.h0[(int64_t)b * H + e] : 0.f;
    hS[0][e] = v;
    hS[1][e] = 0.f;
    if (e < H) a.hbuf[(int64_t)b * H + e] = v;
  }
  __syncthreads();
  tick(0);
  // W_hh: issued now, consumed after the x-part loop
  float w[4][KQ];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float* r = a.w_hh + (int64_t)(j * H + uc) * H + q * KQ;
#pragma unroll
    for (int kk = 0; kk < KQ; kk += 2) {
      float2 v = q * KQ + kk + 1 < H ? *reinterpret_cast<const float2*>(r + kk) : float2{0.f, 0.f};
      w[j][kk] = v.x;
      w[j][kk + 1] = v.y;
    }
  }
  for (int t = 0; t < a.S; ++t) {
    const float4* xp = reinterpret_cast<const float4*>(xS + t * KX + q * XQ);
    float p[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k4 = 0; k4 < XQ / 4; ++k4) {
      const float4 v = xp[k4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        p[j] = fmaf(v.x, wx[j][4 * k4], p[j]);
        p[j] = fmaf(v.y, wx[j][4 * k4 + 1], p[j]);
        p[j] = fmaf(v.z, wx[j][4 * k4 + 2], p[j]);
        p[j] = fmaf(v.w, wx[j][4 * k4 + 3], p[j]);
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      p[j] += qx1(p[j]);
      p[j] += qx2(p[j]);
    }
    const float mine = q == 0 ? p[0] : q == 1 ? p[1] : q == 2 ? p[2] : p[3];
    xP[t * NT + tid] = mine + bh;
  }
  tick(1);
  __builtin_amdgcn_s_waitcnt(0x0F70);     // W_hh landed
  __builtin_amdgcn_s_waitcnt(0xC07F);     // xP stores done (own values only: no barrier)
  tick(2);
  float* hb = a.hbuf + BH + (int64_t)b * H + uc;
  float* cb = a.cbuf + BH + (int64_t)b * H + uc;
  float* gp = a.gates + (int64_t)b * G4 + g;
  const int64_t gstep = (int64_t)B * G4;
  float ph = 0.f, pc = 0.f, pav = 0.f;
  for (int t = 0; t < a.S; ++t) {
    const float* hp = hS[t & 1] + q * KQ;
    float* hn = hS[(t + 1) & 1];
    const float xacc = xP[t * NT + tid];
    const float2* h2 = reinterpret_cast<const float2*>(hp);
    float2 hv[KQ / 2];
#pragma unroll
    for (int i = 0; i < KQ / 2; ++i) hv[i] = h2[i];
    // the previous step's stores, behind this step's LDS reads
    if (t > 0 && act) {
      if (q == 0) {
        hb[0] = ph;
        cb[0] = pc;
        hb += BH;
        cb += BH;
      }
      gp[0] = pav;
      gp += gstep;
    }
    float p[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < KQ / 2; ++i) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        p[j] = fmaf(hv[i].x, w[j][2 * i], p[j]);
        p[j] = fmaf(hv[i].y, w[j][2 * i + 1], p[j]);
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      p[j] += qx1(p[j]);
      p[j] += qx2(p[j]);
    }
    const float mine = q == 0 ? p[0] : q == 1 ? p[1] : q == 2 ? p[2] : p[3];
    const float pre = xacc + mine;
    if (TICKS) __builtin_amdgcn_sched_barrier(0);
    tick(3);
    const float av = q == 2 ? ftanh(pre) : sigm(pre);
    const float ig = quad_bcast<0>(av), fg = quad_bcast<1>(av);
    const float cg = quad_bcast<2>(av), og = quad_bcast<3>(av);
    const float c = fg * creg + ig * cg;
    const float h = og * ftanh(c);
    creg = c;
    if (act && q == 0) hn[u] = h;
    ph = h; pc = c; pav = av;
    if (TICKS) __builtin_amdgcn_sched_barrier(0);
    tick(4);
    __syncthreads();
    tick(5);
  }
  if (a.S > 0 && act) {
    if (q == 0) {
      hb[0] = ph;
      cb[0] = pc;
    }
    gp[0] = pav;
  }
  if (TICKS && b == 0 && (tid & 63) == 0) {
    for (int i = 0; i < 6; ++i) g_ticks2[tid >> 6][i] = tk[i];
  }
}

__device__ unsigned long long g_ticks3[8][8];
// ---------------------------------------------------------------- V3 = V2 with 8 FMA chains per lane (even / odd k per gate)
// V1's K-split, plus: vector weight loads (float2 runs of each lane's k range),
// W_hh loads issued before the x-part loop (in flight while it runs), per-step
// pointers advanced instead of recomputed, and the step's global stores
// (hbuf, cbuf, gates) issued AFTER the barrier, where they overlap the next
// step's LDS reads instead of delaying the barrier.  TICKS: per-wave phase
// cycles into g_ticks2.
template <bool TICKS>
__global__ void __launch_bounds__(NT) v3_kernel(Args a) {
  __shared__ __attribute__((aligned(16))) float hS[2][KP];
  extern __shared__ __attribute__((aligned(16))) float xS[];
  float* xP = xS + ((a.S * KX + 3) & ~3);
  const int B = a.B;
  const int tid = threadIdx.x, u = tid >> 2, q = tid & 3;
  const bool act = u < H;
  const int uc = act ? u : H - 1;
  const int b = blockIdx.x;
  const int64_t BH = (int64_t)B * H;
  unsigned long long tk[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long tp = TICKS ? __builtin_amdgcn_s_memtime() : 0;
  auto tick = [&](int i) {
    if (TICKS) {
      const unsigned long long n = __builtin_amdgcn_s_memtime();
      tk[i] += n - tp;
      tp = n;
    }
  };
  const int g = q * H + uc;
  // W_ih rows j*H + u over x columns [q*XQ, q*XQ + XQ): float2 runs (row
  // stride 168 B, q*XQ*4 = 48q: 8-byte aligned); columns >= DIN read as 0
  float wx[4][XQ];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float* r = a.w_ih + (int64_t)(j * H + uc) * DIN;
#pragma unroll
    for (int kk = 0; kk < XQ; kk += 2) {
      const int k = q * XQ + kk;
      float2 v = k + 1 < DIN ? *reinterpret_cast<const float2*>(r + k) : float2{0.f, 0.f};
      wx[j][kk] = v.x;
      wx[j][kk + 1] = v.y;
    }
  }
  const float bh = a.b_hh[g] + a.b_ih[g];
  for (int e = tid; e < a.S * KX; e += NT) {
    const int t = e / KX, k = e - t * KX;
    xS[e] = k < DIN ? a.x[((int64_t)t * B + b) * a.ldx + k] : 0.f;
  }
  float creg = a.c0[(int64_t)b * H + uc];
  if (act && q == 0) a.cbuf[(int64_t)b * H + u] = creg;
  for (int e = tid; e < KP; e += NT) {
    const float v = e < H ? a.h0[(int64_t)b * H + e] : 0.f;
    hS[0][e] = v;
    hS[1][e] = 0.f;
    if (e < H) a.hbuf[(int64_t)b * H + e] = v;
  }
  __syncthreads();
  tick(0);
  // W_hh: issued now, consumed after the x-part loop
  float w[4][KQ];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float* r = a.w_hh + (int64_t)(j * H + uc) * H + q * KQ;
#pragma unroll
    for (int kk = 0; kk < KQ; kk += 2) {
      float2 v = q * KQ + kk + 1 < H ? *reinterpret_cast<const float2*>(r + kk) : float2{0.f, 0.f};
      w[j][kk] = v.x;
      w[j][kk + 1] = v.y;
    }
  }
  for (int t = 0; t < a.S; ++t) {
    const float4* xp = reinterpret_cast<const float4*>(xS + t * KX + q * XQ);
    float p[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k4 = 0; k4 < XQ / 4; ++k4) {
      const float4 v = xp[k4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        p[j] = fmaf(v.x, wx[j][4 * k4], p[j]);
        p[j] = fmaf(v.y, wx[j][4 * k4 + 1], p[j]);
        p[j] = fmaf(v.z, wx[j][4 * k4 + 2], p[j]);
        p[j] = fmaf(v.w, wx[j][4 * k4 + 3], p[j]);
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      p[j] += qx1(p[j]);
      p[j] += qx2(p[j]);
    }
    const float mine = q == 0 ? p[0] : q == 1 ? p[1] : q == 2 ? p[2] : p[3];
    xP[t * NT + tid] = mine + bh;
  }
  tick(1);
  __builtin_amdgcn_s_waitcnt(0x0F70);     // W_hh landed
  __builtin_amdgcn_s_waitcnt(0xC07F);     // xP stores done (own values only: no barrier)
  tick(2);
  float* hb = a.hbuf + BH + (int64_t)b * H + uc;
  float* cb = a.cbuf + BH + (int64_t)b * H + uc;
  float* gp = a.gates + (int64_t)b * G4 + g;
  const int64_t gstep = (int64_t)B * G4;
  float ph = 0.f, pc = 0.f, pav = 0.f;
  for (int t = 0; t < a.S; ++t) {
    const float* hp = hS[t & 1] + q * KQ;
    float* hn = hS[(t + 1) & 1];
    const float xacc = xP[t * NT + tid];
    const float2* h2 = reinterpret_cast<const float2*>(hp);
    float2 hv[KQ / 2];
#pragma unroll
    for (int i = 0; i < KQ / 2; ++i) hv[i] = h2[i];
    // the previous step's stores, behind this step's LDS reads
    if (t > 0 && act) {
      if (q == 0) {
        hb[0] = ph;
        cb[0] = pc;
        hb += BH;
        cb += BH;
      }
      gp[0] = pav;
      gp += gstep;
    }
    float p[4] = {0.f, 0.f, 0.f, 0.f}, pe[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < KQ / 2; ++i) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        p[j] = fmaf(hv[i].x, w[j][2 * i], p[j]);
        pe[j] = fmaf(hv[i].y, w[j][2 * i + 1], pe[j]);
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      p[j] += pe[j];
      p[j] += qx1(p[j]);
      p[j] += qx2(p[j]);
    }
    const float mine = q == 0 ? p[0] : q == 1 ? p[1] : q == 2 ? p[2] : p[3];
    const float pre = xacc + mine;
    if (TICKS) __builtin_amdgcn_sched_barrier(0);
    tick(3);
    const float av = q == 2 ? ftanh(pre) : sigm(pre);
    const float ig = quad_bcast<0>(av), fg = quad_bcast<1>(av);
    const float cg = quad_bcast<2>(av), og = quad_bcast<3>(av);
    const float c = fg * creg + ig * cg;
    const float h = og * ftanh(c);
    creg = c;
    if (act && q == 0) hn[u] = h;
    ph = h; pc = c; pav = av;
    if (TICKS) __builtin_amdgcn_sched_barrier(0);
    tick(4);
    __syncthreads();
    tick(5);
  }
  if (a.S > 0 && act) {
    if (q == 0) {
      hb[0] = ph;
      cb[0] = pc;
    }
    gp[0] = pav;
  }
  if (TICKS && b == 0 && (tid & 63) == 0) {
    for (int i = 0; i < 6; ++i) g_ticks3[tid >> 6][i] = tk[i];
  }
}

__device__ unsigned long long g_ticks4[8][8];
// ---------------------------------------------------------------- V4 = V3 on v_pk_fma_f32: (even, odd) k pairs as packed lanes
// V1's K-split, plus: vector weight loads (float2 runs of each lane's k range),
// W_hh loads issued before the x-part loop (in flight while it runs), per-step
// pointers advanced instead of recomputed, and the step's global stores
// (hbuf, cbuf, gates) issued AFTER the barrier, where they overlap the next
// step's LDS reads instead of delaying the barrier.  TICKS: per-wave phase
// cycles into g_ticks2.
template <bool TICKS>
__global__ void __launch_bounds__(NT) v4_kernel(Args a) {
  __shared__ __attribute__((aligned(16))) float hS[2][KP];
  extern __shared__ __attribute__((aligned(16))) float xS[];
  float* xP = xS + ((a.S * KX + 3) & ~3);
  const int B = a.B;
  const int tid = threadIdx.x, u = tid >> 2, q = tid & 3;
  const bool act = u < H;
  const int uc = act ? u : H - 1;
  const int b = blockIdx.x;
  const int64_t BH = (int64_t)B * H;
  unsigned long long tk[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long tp = TICKS ? __builtin_amdgcn_s_memtime() : 0;
  auto tick = [&](int i) {
    if (TICKS) {
      const unsigned long long n = __builtin_amdgcn_s_memtime();
      tk[i] += n - tp;
      tp = n;
    }
  };
  const int g = q * H + uc;
  // W_ih rows j*H + u over x columns [q*XQ, q*XQ + XQ): float2 runs (row
  // stride 168 B, q*XQ*4 = 48q: 8-byte aligned); columns >= DIN read as 0
  float wx[4][XQ];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float* r = a.w_ih + (int64_t)(j * H + uc) * DIN;
#pragma unroll
    for (int kk = 0; kk < XQ; kk += 2) {
      const int k = q * XQ + kk;
      float2 v = k + 1 < DIN ? *reinterpret_cast<const float2*>(r + k) : float2{0.f, 0.f};
      wx[j][kk] = v.x;
      wx[j][kk + 1] = v.y;
    }
  }
  const float bh = a.b_hh[g] + a.b_ih[g];
  for (int e = tid; e < a.S * KX; e += NT) {
    const int t = e / KX, k = e - t * KX;
    xS[e] = k < DIN ? a.x[((int64_t)t * B + b) * a.ldx + k] : 0.f;
  }
  float creg = a.c0[(int64_t)b * H + uc];
  if (act && q == 0) a.cbuf[(int64_t)b * H + u] = creg;
  for (int e = tid; e < KP; e += NT) {
    const float v = e < H ? a.h0[(int64_t)b * H + e] : 0.f;
    hS[0][e] = v;
    hS[1][e] = 0.f;
    if (e < H) a.hbuf[(int64_t)b * H + e] = v;
  }
  __syncthreads();
  tick(0);
  // W_hh: issued now, consumed after the x-part loop
  vf2 wv[4][KQ / 2];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float* r = a.w_hh + (int64_t)(j * H + uc) * H + q * KQ;
#pragma unroll
    for (int kk = 0; kk < KQ; kk += 2) {
      float2 v = q * KQ + kk + 1 < H ? *reinterpret_cast<const float2*>(r + kk) : float2{0.f, 0.f};
      wv[j][kk / 2] = vf2{v.x, v.y};
    }
  }
  for (int t = 0; t < a.S; ++t) {
    const float4* xp = reinterpret_cast<const float4*>(xS + t * KX + q * XQ);
    float p[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k4 = 0; k4 < XQ / 4; ++k4) {
      const float4 v = xp[k4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        p[j] = fmaf(v.x, wx[j][4 * k4], p[j]);
        p[j] = fmaf(v.y, wx[j][4 * k4 + 1], p[j]);
        p[j] = fmaf(v.z, wx[j][4 * k4 + 2], p[j]);
        p[j] = fmaf(v.w, wx[j][4 * k4 + 3], p[j]);
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      p[j] += qx1(p[j]);
      p[j] += qx2(p[j]);
    }
    const float mine = q == 0 ? p[0] : q == 1 ? p[1] : q == 2 ? p[2] : p[3];
    xP[t * NT + tid] = mine + bh;
  }
  tick(1);
  __builtin_amdgcn_s_waitcnt(0x0F70);     // W_hh landed
  __builtin_amdgcn_s_waitcnt(0xC07F);     // xP stores done (own values only: no barrier)
  tick(2);
  float* hb = a.hbuf + BH + (int64_t)b * H + uc;
  float* cb = a.cbuf + BH + (int64_t)b * H + uc;
  float* gp = a.gates + (int64_t)b * G4 + g;
  const int64_t gstep = (int64_t)B * G4;
  float ph = 0.f, pc = 0.f, pav = 0.f;
  for (int t = 0; t < a.S; ++t) {
    const float* hp = hS[t & 1] + q * KQ;
    float* hn = hS[(t + 1) & 1];
    const float xacc = xP[t * NT + tid];
    const float2* h2 = reinterpret_cast<const float2*>(hp);
    float2 hv[KQ / 2];
#pragma unroll
    for (int i = 0; i < KQ / 2; ++i) hv[i] = h2[i];
    // the previous step's stores, behind this step's LDS reads
    if (t > 0 && act) {
      if (q == 0) {
        hb[0] = ph;
        cb[0] = pc;
        hb += BH;
        cb += BH;
      }
      gp[0] = pav;
      gp += gstep;
    }
    vf2 pp[4] = {vf2{0.f, 0.f}, vf2{0.f, 0.f}, vf2{0.f, 0.f}, vf2{0.f, 0.f}};
#pragma unroll
    for (int i = 0; i < KQ / 2; ++i) {
      const vf2 h2v = vf2{hv[i].x, hv[i].y};
#pragma unroll
      for (int j = 0; j < 4; ++j) pp[j] = __builtin_elementwise_fma(h2v, wv[j][i], pp[j]);
    }
    float p[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      p[j] = pp[j].x + pp[j].y;
      p[j] += qx1(p[j]);
      p[j] += qx2(p[j]);
    }
    const float mine = q == 0 ? p[0] : q == 1 ? p[1] : q == 2 ? p[2] : p[3];
    const float pre = xacc + mine;
    if (TICKS) __builtin_amdgcn_sched_barrier(0);
    tick(3);
    const float av = q == 2 ? ftanh(pre) : sigm(pre);
    const float ig = quad_bcast<0>(av), fg = quad_bcast<1>(av);
    const float cg = quad_bcast<2>(av), og = quad_bcast<3>(av);
    const float c = fg * creg + ig * cg;
    const float h = og * ftanh(c);
    creg = c;
    if (act && q == 0) hn[u] = h;
    ph = h; pc = c; pav = av;
    if (TICKS) __builtin_amdgcn_sched_barrier(0);
    tick(4);
    __syncthreads();
    tick(5);
  }
  if (a.S > 0 && act) {
    if (q == 0) {
      hb[0] = ph;
      cb[0] = pc;
    }
    gp[0] = pav;
  }
  if (TICKS && b == 0 && (tid & 63) == 0) {
    for (int i = 0; i < 6; ++i) g_ticks4[tid >> 6][i] = tk[i];
  }
}

__device__ unsigned long long g_ticks5[8][8];
// ---------------------------------------------------------------- V5 = V4 with the units dealt over 8 waves (wave w: units w, w+8, ...; 13 per wave) so each SIMD's two waves carry 25 units, not 32
// V1's K-split, plus: vector weight loads (float2 runs of each lane's k range),
// W_hh loads issued before the x-part loop (in flight while it runs), per-step
// pointers advanced instead of recomputed, and the step's global stores
// (hbuf, cbuf, gates) issued AFTER the barrier, where they overlap the next
// step's LDS reads instead of delaying the barrier.  TICKS: per-wave phase
// cycles into g_ticks2.
template <bool TICKS>
__global__ void __launch_bounds__(512) v5_kernel(Args a) {
  __shared__ __attribute__((aligned(16))) float hS[2][KP];
  extern __shared__ __attribute__((aligned(16))) float xS[];
  float* xP = xS + ((a.S * KX + 3) & ~3);
  const int B = a.B;
  const int tid = threadIdx.x, lane = tid & 63, wv_ = tid >> 6;
  const int u = (lane >> 2) * 8 + wv_, q = lane & 3;
  const bool act = (lane >> 2) < 13 && u < H;
  const int uc = act ? u : H - 1;
  const int b = blockIdx.x;
  const int64_t BH = (int64_t)B * H;
  unsigned long long tk[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long tp = TICKS ? __builtin_amdgcn_s_memtime() : 0;
  auto tick = [&](int i) {
    if (TICKS) {
      const unsigned long long n = __builtin_amdgcn_s_memtime();
      tk[i] += n - tp;
      tp = n;
    }
  };
  const int g = q * H + uc;
  // W_ih rows j*H + u over x columns [q*XQ, q*XQ + XQ): float2 runs (row
  // stride 168 B, q*XQ*4 = 48q: 8-byte aligned); columns >= DIN read as 0
  float wx[4][XQ];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float* r = a.w_ih + (int64_t)(j * H + uc) * DIN;
#pragma unroll
    for (int kk = 0; kk < XQ; kk += 2) {
      const int k = q * XQ + kk;
      float2 v = k + 1 < DIN ? *reinterpret_cast<const float2*>(r + k) : float2{0.f, 0.f};
      wx[j][kk] = v.x;
      wx[j][kk + 1] = v.y;
    }
  }
  const float bh = a.b_hh[g] + a.b_ih[g];
  for (int e = tid; e < a.S * KX; e += 512) {
    const int t = e / KX, k = e - t * KX;
    xS[e] = k < DIN ? a.x[((int64_t)t * B + b) * a.ldx + k] : 0.f;
  }
  float creg = a.c0[(int64_t)b * H + uc];
  if (act && q == 0) a.cbuf[(int64_t)b * H + u] = creg;
  for (int e = tid; e < KP; e += 512) {
    const float v = e < H ? a.h0[(int64_t)b * H + e] : 0.f;
    hS[0][e] = v;
    hS[1][e] = 0.f;
    if (e < H) a.hbuf[(int64_t)b * H + e] = v;
  }
  __syncthreads();
  tick(0);
  // W_hh: issued now, consumed after the x-part loop
  vf2 wv[4][KQ / 2];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float* r = a.w_hh + (int64_t)(j * H + uc) * H + q * KQ;
#pragma unroll
    for (int kk = 0; kk < KQ; kk += 2) {
      float2 v = q * KQ + kk + 1 < H ? *reinterpret_cast<const float2*>(r + kk) : float2{0.f, 0.f};
      wv[j][kk / 2] = vf2{v.x, v.y};
    }
  }
  for (int t = 0; t < a.S; ++t) {
    const float4* xp = reinterpret_cast<const float4*>(xS + t * KX + q * XQ);
    float p[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k4 = 0; k4 < XQ / 4; ++k4) {
      const float4 v = xp[k4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        p[j] = fmaf(v.x, wx[j][4 * k4], p[j]);
        p[j] = fmaf(v.y, wx[j][4 * k4 + 1], p[j]);
        p[j] = fmaf(v.z, wx[j][4 * k4 + 2], p[j]);
        p[j] = fmaf(v.w, wx[j][4 * k4 + 3], p[j]);
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      p[j] += qx1(p[j]);
      p[j] += qx2(p[j]);
    }
    const float mine = q == 0 ? p[0] : q == 1 ? p[1] : q == 2 ? p[2] : p[3];
    xP[t * 512 + tid] = mine + bh;
  }
  tick(1);
  __builtin_amdgcn_s_waitcnt(0x0F70);     // W_hh landed
  __builtin_amdgcn_s_waitcnt(0xC07F);     // xP stores done (own values only: no barrier)
  tick(2);
  float* hb = a.hbuf + BH + (int64_t)b * H + uc;
  float* cb = a.cbuf + BH + (int64_t)b * H + uc;
  float* gp = a.gates + (int64_t)b * G4 + g;
  const int64_t gstep = (int64_t)B * G4;
  float ph = 0.f, pc = 0.f, pav = 0.f;
  for (int t = 0; t < a.S; ++t) {
    const float* hp = hS[t & 1] + q * KQ;
    float* hn = hS[(t + 1) & 1];
    const float xacc = xP[t * 512 + tid];
    const float2* h2 = reinterpret_cast<const float2*>(hp);
    float2 hv[KQ / 2];
#pragma unroll
    for (int i = 0; i < KQ / 2; ++i) hv[i] = h2[i];
    // the previous step's stores, behind this step's LDS reads
    if (t > 0 && act) {
      if (q == 0) {
        hb[0] = ph;
        cb[0] = pc;
        hb += BH;
        cb += BH;
      }
      gp[0] = pav;
      gp += gstep;
    }
    vf2 pp[4] = {vf2{0.f, 0.f}, vf2{0.f, 0.f}, vf2{0.f, 0.f}, vf2{0.f, 0.f}};
#pragma unroll
    for (int i = 0; i < KQ / 2; ++i) {
      const vf2 h2v = vf2{hv[i].x, hv[i].y};
#pragma unroll
      for (int j = 0; j < 4; ++j) pp[j] = __builtin_elementwise_fma(h2v, wv[j][i], pp[j]);
    }
    float p[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      p[j] = pp[j].x + pp[j].y;
      p[j] += qx1(p[j]);
      p[j] += qx2(p[j]);
    }
    const float mine = q == 0 ? p[0] : q == 1 ? p[1] : q == 2 ? p[2] : p[3];
    const float pre = xacc + mine;
    if (TICKS) __builtin_amdgcn_sched_barrier(0);
    tick(3);
    const float av = q == 2 ? ftanh(pre) : sigm(pre);
    const float ig = quad_bcast<0>(av), fg = quad_bcast<1>(av);
    const float cg = quad_bcast<2>(av), og = quad_bcast<3>(av);
    const float c = fg * creg + ig * cg;
    const float h = og * ftanh(c);
    creg = c;
    if (act && q == 0) hn[u] = h;
    ph = h; pc = c; pav = av;
    if (TICKS) __builtin_amdgcn_sched_barrier(0);
    tick(4);
    __syncthreads();
    tick(5);
  }
  if (a.S > 0 && act) {
    if (q == 0) {
      hb[0] = ph;
      cb[0] = pc;
    }
    gp[0] = pav;
  }
  if (TICKS && b == 0 && (tid & 63) == 0) {
    for (int i = 0; i < 6; ++i) g_ticks5[tid >> 6][i] = tk[i];
  }
}

// ================================================================ BPTT
struct BArgs {
  const float* dh; const float* gates; const float* cbuf; const float* w_hh; int S, B;
  float* dgates;
};
// B0: the product's lstm_bwd_v_kernel<1, 104>
__global__ void __launch_bounds__(NT) b0_kernel(BArgs a) {
  constexpr int R = 1;
  __shared__ __attribute__((aligned(16))) float dG[2][R * 4 * KP];
  const int B = a.B;
  const int tid = threadIdx.x, u = tid >> 2, q = tid & 3;
  const bool act = u < H;
  const int uc = act ? u : H - 1;
  const int g = q * H + uc;
  const int r0 = blockIdx.x * R;
  const int64_t BH = (int64_t)B * H;
  for (int e = tid; e < 2 * R * 4 * KP; e += NT) (&dG[0][0])[e] = 0.f;
  float w[KP];
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
  struct In { float gq[R], ct[R], ctm[R], dho[R]; };
  In A, Bn;
  float dcreg[R], dhr[R];
  auto fetch = [&](int t, In& X) {
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
      v_dot_pipelined(dp, w, s0, s1, s2, s3);
      const float p = (s0 + s1) + (s2 + s3);
      dhr[r] = (quad_bcast<0>(p) + quad_bcast<1>(p)) + (quad_bcast<2>(p) + quad_bcast<3>(p));
    }
    return true;
  };
  for (int t = a.S - 1; t >= 0; t -= 2) {
    if (!step(t, A)) break;
    if (!step(t - 1, Bn)) break;
  }
}

// B1: the recurrent product dh_rec = dgates_t W_hh with K split over the 16
// lanes of a row: lane (ug = tid >> 4, rr = tid & 15) holds W_hh[r][4ug..4ug+3]
// for rows r in [25 rr, 25 rr + 25) (one float4 per row), reads those 25
// dgates (7 ds_read_b128 of a [16][28]-padded image) and sums its 4 units;
// the 16 partials of a unit meet through 4 DPP adds (quad xor 1, xor 2, row
// half-mirror, row rotate 8: every lane of the row ends with the same sums).
// The cell backward keeps the (u, q) = (tid >> 2, tid & 3) mapping: unit u's
// sum sits in its own row at index (tid >> 2) & 3.
constexpr int BR = 25, BRP = 28;
__device__ __forceinline__ float hmirror(float v) {   // row_half_mirror
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x141, 0xF, 0xF, false));
}
__device__ __forceinline__ float ror8(float v) {      // row_ror:8
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x128, 0xF, 0xF, false));
}
__global__ void __launch_bounds__(NT) b1_kernel(BArgs a) {
  __shared__ __attribute__((aligned(16))) float dG[2][16 * BRP];
  const int B = a.B;
  const int tid = threadIdx.x, u = tid >> 2, q = tid & 3;
  const bool act = u < H;
  const int uc = act ? u : H - 1;
  const int g = q * H + uc;
  const int b = blockIdx.x;
  const int64_t BH = (int64_t)B * H;
  const int ug = tid >> 4, rr = tid & 15;
  const int ugc = ug < H / 4 ? ug : H / 4 - 1;
  for (int e = tid; e < 2 * 16 * BRP; e += NT) (&dG[0][0])[e] = 0.f;
  float4 w[BR];
#pragma unroll
  for (int i = 0; i < BR; ++i)
    w[i] = *reinterpret_cast<const float4*>(a.w_hh + (int64_t)(rr * BR + i) * H + 4 * ugc);
  const int dgi = (g / BR) * BRP + g % BR;        // this lane's dgate in the padded image
  float gq = 0.f, ct = 0.f, ctm = 0.f, dho = 0.f, gqn, ctn, ctmn, dhon;
  auto fetch = [&](int t, float& G, float& C, float& CM, float& DH) {
    G = a.gates[((int64_t)t * B + b) * G4 + g];
    C = a.cbuf[(int64_t)(t + 1) * BH + (int64_t)b * H + uc];
    CM = a.cbuf[(int64_t)t * BH + (int64_t)b * H + uc];
    DH = a.dh[(int64_t)t * BH + (int64_t)b * H + uc];
  };
  if (a.S <= 0) return;
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
    if (act) dgw[dgi] = dq;
    if (act) a.dgates[((int64_t)t * B + b) * G4 + g] = dq;
    gq = gqn; ct = ctn; ctm = ctmn; dho = dhon;
    fetch(t >= 2 ? t - 2 : 0, gqn, ctn, ctmn, dhon);
    __syncthreads();
    if (t == 0) break;
    const float4* dp = reinterpret_cast<const float4*>(dgw + rr * BRP);
    float4 dv[BRP / 4];
#pragma unroll
    for (int i = 0; i < BRP / 4; ++i) dv[i] = dp[i];
    float p0 = 0.f, p1 = 0.f, p2 = 0.f, p3 = 0.f;
#pragma unroll
    for (int i = 0; i < BR; ++i) {
      const float d = (i & 3) == 0 ? dv[i >> 2].x : (i & 3) == 1 ? dv[i >> 2].y : (i & 3) == 2 ? dv[i >> 2].z : dv[i >> 2].w;
      p0 = fmaf(d, w[i].x, p0);
      p1 = fmaf(d, w[i].y, p1);
      p2 = fmaf(d, w[i].z, p2);
      p3 = fmaf(d, w[i].w, p3);
    }
    p0 += qx1(p0); p1 += qx1(p1); p2 += qx1(p2); p3 += qx1(p3);
    p0 += qx2(p0); p1 += qx2(p1); p2 += qx2(p2); p3 += qx2(p3);
    p0 += hmirror(p0); p1 += hmirror(p1); p2 += hmirror(p2); p3 += hmirror(p3);
    p0 += ror8(p0); p1 += ror8(p1); p2 += ror8(p2); p3 += ror8(p3);
    const int k = (tid >> 2) & 3;
    dhr = k == 0 ? p0 : k == 1 ? p1 : k == 2 ? p2 : p3;
  }
}

__global__ void __launch_bounds__(512) b3_kernel(BArgs a) {
  __shared__ __attribute__((aligned(16))) float dG[2][16 * BRP];
  const int B = a.B;
  const int tid = threadIdx.x, lane = tid & 63, wv_ = tid >> 6;
  const int ug = (lane >> 4) * 8 + wv_, rr = lane & 15;       // row group of 16 lanes
  const int u = 4 * ug + (rr >> 2), q = rr & 3;
  const bool act = u < H;
  const int uc = act ? u : H - 1;
  const int g = q * H + uc;
  const int b = blockIdx.x;
  const int64_t BH = (int64_t)B * H;
  const int ugc = ug < H / 4 ? ug : H / 4 - 1;
  for (int e = tid; e < 2 * 16 * BRP; e += 512) (&dG[0][0])[e] = 0.f;
  float4 w[BR];
#pragma unroll
  for (int i = 0; i < BR; ++i)
    w[i] = *reinterpret_cast<const float4*>(a.w_hh + (int64_t)(rr * BR + i) * H + 4 * ugc);
  const int dgi = (g / BR) * BRP + g % BR;        // this lane's dgate in the padded image
  float gq = 0.f, ct = 0.f, ctm = 0.f, dho = 0.f, gqn, ctn, ctmn, dhon;
  auto fetch = [&](int t, float& G, float& C, float& CM, float& DH) {
    G = a.gates[((int64_t)t * B + b) * G4 + g];
    C = a.cbuf[(int64_t)(t + 1) * BH + (int64_t)b * H + uc];
    CM = a.cbuf[(int64_t)t * BH + (int64_t)b * H + uc];
    DH = a.dh[(int64_t)t * BH + (int64_t)b * H + uc];
  };
  if (a.S <= 0) return;
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
    if (act) dgw[dgi] = dq;
    if (act) a.dgates[((int64_t)t * B + b) * G4 + g] = dq;
    gq = gqn; ct = ctn; ctm = ctmn; dho = dhon;
    fetch(t >= 2 ? t - 2 : 0, gqn, ctn, ctmn, dhon);
    __syncthreads();
    if (t == 0) break;
    const float4* dp = reinterpret_cast<const float4*>(dgw + rr * BRP);
    float4 dv[BRP / 4];
#pragma unroll
    for (int i = 0; i < BRP / 4; ++i) dv[i] = dp[i];
    float p0 = 0.f, p1 = 0.f, p2 = 0.f, p3 = 0.f;
#pragma unroll
    for (int i = 0; i < BR; ++i) {
      const float d = (i & 3) == 0 ? dv[i >> 2].x : (i & 3) == 1 ? dv[i >> 2].y : (i & 3) == 2 ? dv[i >> 2].z : dv[i >> 2].w;
      p0 = fmaf(d, w[i].x, p0);
      p1 = fmaf(d, w[i].y, p1);
      p2 = fmaf(d, w[i].z, p2);
      p3 = fmaf(d, w[i].w, p3);
    }
    p0 += qx1(p0); p1 += qx1(p1); p2 += qx1(p2); p3 += qx1(p3);
    p0 += qx2(p0); p1 += qx2(p1); p2 += qx2(p2); p3 += qx2(p3);
    p0 += hmirror(p0); p1 += hmirror(p1); p2 += hmirror(p2); p3 += hmirror(p3);
    p0 += ror8(p0); p1 += ror8(p1); p2 += ror8(p2); p3 += ror8(p3);
    const int k = (rr >> 2) & 3;
    dhr = k == 0 ? p0 : k == 1 ? p1 : k == 2 ? p2 : p3;
  }
}

__global__ void __launch_bounds__(NT) b2_kernel(BArgs a) {
  __shared__ __attribute__((aligned(16))) float dG[2][16 * BRP];
  const int B = a.B;
  const int tid = threadIdx.x, u = tid >> 2, q = tid & 3;
  const bool act = u < H;
  const int uc = act ? u : H - 1;
  const int g = q * H + uc;
  const int b = blockIdx.x;
  const int64_t BH = (int64_t)B * H;
  const int ug = tid >> 4, rr = tid & 15;
  const int ugc = ug < H / 4 ? ug : H / 4 - 1;
  for (int e = tid; e < 2 * 16 * BRP; e += NT) (&dG[0][0])[e] = 0.f;
  float4 w[BR];
#pragma unroll
  for (int i = 0; i < BR; ++i)
    w[i] = *reinterpret_cast<const float4*>(a.w_hh + (int64_t)(rr * BR + i) * H + 4 * ugc);
  const int dgi = (g / BR) * BRP + g % BR;        // this lane's dgate in the padded image
  float gq = 0.f, ct = 0.f, ctm = 0.f, dho = 0.f, gqn, ctn, ctmn, dhon;
  auto fetch = [&](int t, float& G, float& C, float& CM, float& DH) {
    G = a.gates[((int64_t)t * B + b) * G4 + g];
    C = a.cbuf[(int64_t)(t + 1) * BH + (int64_t)b * H + uc];
    CM = a.cbuf[(int64_t)t * BH + (int64_t)b * H + uc];
    DH = a.dh[(int64_t)t * BH + (int64_t)b * H + uc];
  };
  if (a.S <= 0) return;
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
    if (act) dgw[dgi] = dq;
    if (act) a.dgates[((int64_t)t * B + b) * G4 + g] = dq;
    gq = gqn; ct = ctn; ctm = ctmn; dho = dhon;
    fetch(t >= 2 ? t - 2 : 0, gqn, ctn, ctmn, dhon);
    __syncthreads();
    if (t == 0) break;
    const float4* dp = reinterpret_cast<const float4*>(dgw + rr * BRP);
    float4 dv[BRP / 4];
#pragma unroll
    for (int i = 0; i < BRP / 4; ++i) dv[i] = dp[i];
    vf2 p01 = {0.f, 0.f}, p23 = {0.f, 0.f};
#pragma unroll
    for (int i = 0; i < BR; ++i) {
      const float d = (i & 3) == 0 ? dv[i >> 2].x : (i & 3) == 1 ? dv[i >> 2].y : (i & 3) == 2 ? dv[i >> 2].z : dv[i >> 2].w;
      p01 = __builtin_elementwise_fma(vf2{d, d}, vf2{w[i].x, w[i].y}, p01);
      p23 = __builtin_elementwise_fma(vf2{d, d}, vf2{w[i].z, w[i].w}, p23);
    }
    float p0 = p01.x, p1 = p01.y, p2 = p23.x, p3 = p23.y;
    p0 += qx1(p0); p1 += qx1(p1); p2 += qx1(p2); p3 += qx1(p3);
    p0 += qx2(p0); p1 += qx2(p1); p2 += qx2(p2); p3 += qx2(p3);
    p0 += hmirror(p0); p1 += hmirror(p1); p2 += hmirror(p2); p3 += hmirror(p3);
    p0 += ror8(p0); p1 += ror8(p1); p2 += ror8(p2); p3 += ror8(p3);
    const int k = (tid >> 2) & 3;
    dhr = k == 0 ? p0 : k == 1 ? p1 : k == 2 ? p2 : p3;
  }
}

typedef void (*BFn)(BArgs);
static float runb(BFn k, const BArgs& a, int iters, int nt = NT) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<float> ts;
  for (int i = 0; i < iters + 3; ++i) {
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(k, dim3(a.B), dim3(nt), 0, 0, a);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (i >= 3) ts.push_back(ms * 1e3f);
  }
  std::sort(ts.begin(), ts.end());
  return ts[ts.size() / 2];
}

typedef void (*KFn)(Args);

static float run(KFn k, const Args& a, int iters, int nt = NT, size_t min_lds = 0) {
  size_t lds = ((size_t)((a.S * KX + 3) & ~3) + (size_t)a.S * nt) * 4;
  if (lds < min_lds) lds = min_lds;
  CK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<float> ts;
  for (int i = 0; i < iters + 3; ++i) {
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(k, dim3(a.B), dim3(nt), lds, 0, a);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (i >= 3) ts.push_back(ms * 1e3f);
  }
  std::sort(ts.begin(), ts.end());
  return ts[ts.size() / 2];
}

int main() {
  const int B = 128, SMAX = 41;
  const int ldx = DIN;
  std::vector<float> hx((size_t)SMAX * B * ldx), hwih((size_t)G4 * DIN), hbih(G4), hwhh((size_t)G4 * H),
      hbhh(G4), hh0((size_t)B * H), hc0((size_t)B * H);
  srand(1);
  auto rnd = [] { return (float)rand() / RAND_MAX * 2.f - 1.f; };
  for (auto& v : hx) v = rnd();
  for (auto& v : hwih) v = 0.15f * rnd();
  for (auto& v : hwhh) v = 0.1f * rnd();
  for (auto& v : hbih) v = 0.1f * rnd();
  for (auto& v : hbhh) v = 0.1f * rnd();
  for (auto& v : hh0) v = 0.1f * rnd();
  for (auto& v : hc0) v = 0.1f * rnd();
  auto up = [](const std::vector<float>& h) {
    float* d;
    CK(hipMalloc(&d, h.size() * 4));
    CK(hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    return d;
  };
  float *dx = up(hx), *dwih = up(hwih), *dbih = up(hbih), *dwhh = up(hwhh), *dbhh = up(hbhh),
        *dh0 = up(hh0), *dc0 = up(hc0);
  float *hb[2], *cb[2], *gt[2];
  for (int i = 0; i < 2; ++i) {
    CK(hipMalloc(&hb[i], (size_t)(SMAX + 1) * B * H * 4));
    CK(hipMalloc(&cb[i], (size_t)(SMAX + 1) * B * H * 4));
    CK(hipMalloc(&gt[i], (size_t)SMAX * B * G4 * 4));
  }
  KFn ks[5] = {v0_kernel, v4_kernel<false>, v5_kernel<false>, v5_kernel<true>, v4_kernel<true>};
  const char* names[5] = {"V0", "V4", "V5", "V5t", "V4t"};
  const int Ss[3] = {1, 21, 41};
  for (int v = 0; v < 5; ++v) {
    float t[3];
    for (int si = 0; si < 3; ++si) {
      Args a{dx, ldx, dwih, dbih, dwhh, dbhh, dh0, dc0, Ss[si], B, hb[v ? 1 : 0], cb[v ? 1 : 0], gt[v ? 1 : 0]};
      t[si] = run(ks[v], a, 30, (v == 2 || v == 3) ? 512 : NT);
    }
    printf("{\"variant\": \"%s\", \"us_S1\": %.2f, \"us_S21\": %.2f, \"us_S41\": %.2f, \"us_per_step\": %.3f}\n",
           names[v], t[0], t[1], t[2], (t[2] - t[0]) / 40.f);
  }
  {   // co-residence: segments per launch 128 / 32 / 1, and 128 with 96 KB of
      // dynamic LDS (one workgroup per CU)
    struct Co { int B; size_t lds; } co[4] = {{128, 0}, {32, 0}, {1, 0}, {128, 96 * 1024}};
    for (int kv = 0; kv < 2; ++kv)
    for (auto& c : co) {
      float t[3];
      for (int si = 0; si < 3; ++si) {
        Args a{dx, ldx, dwih, dbih, dwhh, dbhh, dh0, dc0, Ss[si], c.B, hb[0], cb[0], gt[0]};
        t[si] = run(kv ? v4_kernel<false> : v0_kernel, a, 30, NT, c.lds);
      }
      printf("{\"coresidence\": \"V%d B=%d lds=%zu\", \"us_S1\": %.2f, \"us_S41\": %.2f, \"us_per_step\": %.3f}\n",
             kv ? 4 : 0, c.B, c.lds, t[0], t[2], (t[2] - t[0]) / 40.f);
    }
  }
  {   // phase ticks of V3t at S = 21 (shader cycles per launch, per wave; steps summed)
    Args a{dx, ldx, dwih, dbih, dwhh, dbhh, dh0, dc0, 21, B, hb[1], cb[1], gt[1]};
    run(v5_kernel<true>, a, 1, 512);
    unsigned long long tk[8][8];
    CK(hipMemcpyFromSymbol(tk, HIP_SYMBOL(g_ticks5), sizeof(tk)));
    for (int w = 0; w < 8; ++w)
      printf("{\"v5_ticks_wave\": %d, \"load_stage\": %llu, \"xpart\": %llu, \"whh_wait\": %llu, \"dot_per_step\": %.0f, \"cell_per_step\": %.0f, \"barrier_per_step\": %.0f}\n",
             w, tk[w][0], tk[w][1], tk[w][2], tk[w][3] / 21.0, tk[w][4] / 21.0, tk[w][5] / 21.0);
  }
  // correctness at S = 41: V1 vs V0
  auto dl = [](const float* d, size_t n) {
    std::vector<float> h(n);
    CK(hipMemcpy(h.data(), d, n * 4, hipMemcpyDeviceToHost));
    return h;
  };
  {   // V2t phase ticks at S = 21
    Args a{dx, ldx, dwih, dbih, dwhh, dbhh, dh0, dc0, 21, B, hb[1], cb[1], gt[1]};
    run(v2_kernel<true>, a, 1);
    unsigned long long tk[8][8];
    CK(hipMemcpyFromSymbol(tk, HIP_SYMBOL(g_ticks2), sizeof(tk)));
    for (int w = 0; w < 7; ++w)
      printf("{\"v2_ticks_wave\": %d, \"load_stage\": %llu, \"xpart\": %llu, \"whh_wait\": %llu, \"dot_per_step\": %.0f, \"cell_per_step\": %.0f, \"barrier_per_step\": %.0f}\n",
             w, tk[w][0], tk[w][1], tk[w][2], tk[w][3] / 21.0, tk[w][4] / 21.0, tk[w][5] / 21.0);
  }
  for (int v = 1; v <= 2; ++v) {   // correctness at S = 41: V1 and V2 vs V0
    Args a{dx, ldx, dwih, dbih, dwhh, dbhh, dh0, dc0, SMAX, B, hb[1], cb[1], gt[1]};
    run(v == 1 ? v4_kernel<false> : v5_kernel<false>, a, 1, v == 1 ? NT : 512);
  const size_t nh = (size_t)(SMAX + 1) * B * H, ng = (size_t)SMAX * B * G4;
  auto h0v = dl(hb[0], nh), h1v = dl(hb[1], nh), c0v = dl(cb[0], nh), c1v = dl(cb[1], nh),
       g0v = dl(gt[0], ng), g1v = dl(gt[1], ng);
  double dh = 0, dc = 0, dg = 0;
  for (size_t i = 0; i < nh; ++i) {
    dh = std::max(dh, (double)fabsf(h0v[i] - h1v[i]));
    dc = std::max(dc, (double)fabsf(c0v[i] - c1v[i]));
  }
  for (size_t i = 0; i < ng; ++i) dg = std::max(dg, (double)fabsf(g0v[i] - g1v[i]));
 printf("{\"check\": \"V%d vs V0 at S=41\", \"max_dh\": %.3g, \"max_dc\": %.3g, \"max_dgates\": %.3g}\n", v + 1, dh, dc, dg);
  }
  {   // BPTT: B0 vs B1 at S = 1 / 21 / 41 (inputs: the forward's gates / cbuf, random dh)
    std::vector<float> hdh((size_t)SMAX * B * H);
    for (auto& v : hdh) v = 0.1f * rnd();
    float* ddh = up(hdh);
    float* dg[3];
    for (int i = 0; i < 3; ++i) CK(hipMalloc(&dg[i], (size_t)SMAX * B * G4 * 4));
    BFn bk[3] = {b0_kernel, b1_kernel, b3_kernel};
    for (int v = 0; v < 3; ++v) {
      float t[3];
      for (int si = 0; si < 3; ++si) {
        BArgs ba{ddh, gt[0], cb[0], dwhh, Ss[si], B, dg[v]};
        t[si] = runb(bk[v], ba, 30, v == 2 ? 512 : NT);
      }
      printf("{\"variant\": \"B%d\", \"us_S1\": %.2f, \"us_S21\": %.2f, \"us_S41\": %.2f, \"us_per_step\": %.3f}\n",
             v, t[0], t[1], t[2], (t[2] - t[0]) / 40.f);
    }
    const size_t ng = (size_t)SMAX * B * G4;
    auto d0 = dl(dg[0], ng), d1 = dl(dg[1], ng), d2 = dl(dg[2], ng);
    double md = 0, md2 = 0, mx = 0;
    for (size_t i = 0; i < ng; ++i) {
      md = std::max(md, (double)fabsf(d0[i] - d1[i]));
      md2 = std::max(md2, (double)fabsf(d0[i] - d2[i]));
      mx = std::max(mx, (double)fabsf(d0[i]));
    }
    printf("{\"check\": \"B1 / B3 vs B0 at S=41\", \"max_ddgates\": %.3g, \"max_ddgates_b2\": %.3g, \"max_dgates\": %.3g}\n", md, md2, mx);
  }
  return 0;
}
