// EXPERIMENT (not built; kept for the record, DESIGN.md §6 A/B log).
// Fused three-layer PPO head passes, C3 on one MI355X (bench.py, same box):
//   layer GEMMs (product):          forward  85 us, input-gradient chain 100 us
//   this file, k-loops unrolled:    forward 129 us, backward 132 us  (C3 9.64 -> 11.55 ms)
//   k-loops not unrolled (`in` in private memory): forward 412 us    (C3 21.6 ms)
// Gradients were within the fp64 envelope (tests/test_gpu_parity_pinned.py
// first-step test).  Likely limits: ~100 KB of straight-line MFMA code per
// kernel (instruction cache), 336 row panels on 256 CUs, and a barrier per
// 16-k weight chunk.  Not pursued further this round.
// head_kernels.hip — the PPO actor / critic heads (builders.py:86-175:
// Linear-ReLU-Linear-ReLU-Linear[-Tanh]) as ONE kernel per pass over a row
// panel, for the learner's tall activations (rows = segments x steps).
//
// Forward:   HA1 = relu(X W1^T + b1), HA2 = relu(HA1 W2^T + b2), Y = act(HA2 W3^T + b3)
// Backward:  dH2 = (dZ W3) * [HA2 > 0], dH1 = (dH2 W2) * [HA1 > 0],
//            dX[:, c] = (dH1 W1)[:, dx0 + c] (* [mask > 0])
// (the weight gradients of the three layers are grouped GEMMs elsewhere; this
// pass writes the dH2 / dH1 they read).
//
// Layout trick: a wave owns 16 rows and keeps them as the MFMA's N index; the
// output features are the M index (v_mfma_f32_16x16x4_f32: A(m = li, k = lk),
// B(k = lk, n = li), D(m = 4 lk + r, n = li)).  A lane's accumulator tile t
// therefore holds features 16t + 4lk + r of its row — exactly the B operand of
// the NEXT layer's k-step (t, r) when that layer's k order is permuted the same
// way (slot lk of k-step (t, r) is input feature 16t + 4lk + r; the weight
// chunk in LDS is read with the same permutation, one 16-byte read per 4
// MFMAs).  Activations never leave registers between layers; each layer's
// output is written once (HA1 / HA2 / dH2 / dH1 are needed by the backward /
// the weight gradients).  Weights stream through LDS in 16-k chunks shared by
// the four waves (register prefetch of the next chunk, one barrier per chunk).
// Versus three layer GEMMs: two launches and two HBM round trips of the
// intermediate activations fewer, and the input-gradient chain no longer
// serialises three small launches.
#include "smi_device.hpp"
#include "smi_internal.hpp"

namespace smi {

constexpr int HK_LD = 20;                // LDS row stride of a staged chunk (floats)

struct HeadFwdArgs {
  const float* X; int64_t ldx; int K0;   // input rows [rows][ldx], K0 features
  const float* W1; const float* b1;      // [h1][K0]
  const float* W2; const float* b2;      // [h2][h1]
  const float* W3; const float* b3;      // [out][h2]
  int h1, h2, out, tanh_out;
  float* HA1; float* HA2;                // [rows][h1], [rows][h2]
  float* Y; int64_t ldy;                 // [rows][ldy]
  int64_t rows; const int* skip;
};

struct HeadBwdArgs {
  const float* dZ; int64_t ldz; int out; // gradient at the last layer's pre-activation
  const float* W1; int in;               // [h1][in]
  const float* W2; const float* W3;      // [h2][h1], [out][h2]
  int h1, h2;
  const float* HA1; const float* HA2;    // forward activations (ReLU masks)
  float* dH2; float* dH1;                // [rows][h2], [rows][h1]
  float* dX; int64_t lddx; int dx0, dxn; // input-gradient columns [dx0, dx0 + dxn)
  const float* mask; int64_t ldm;        // optional: dX zero where mask <= 0
  int64_t rows; const int* skip;
};

// One 16-k chunk of a weight matrix for output features m < 16T:
// dst[m*HK_LD + kk] = W(m, kb + kk), zero for m >= M or k >= K.
// KMAJ: W(m, k) = W[m*ldw + k] (forward weights, k contiguous);
// else W(m, k) = W[k*ldw + m] (the transposed view of the backward).
template <int T, bool KMAJ>
struct Stager {
  static constexpr int N = 16 * T * 16;
  static constexpr int PER = (N + kWG - 1) / kWG;
  float v[PER];
  __device__ __forceinline__ void load(const float* __restrict__ W, int64_t ldw, int M, int K,
                                       int kb) {
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const int idx = threadIdx.x + q * kWG;
      int m, kk;
      if constexpr (KMAJ) { m = idx >> 4; kk = idx & 15; }
      else { kk = idx / (16 * T); m = idx - kk * (16 * T); }
      const int k = kb + kk;
      const bool ok = idx < N && m < M && k < K;
      const float* src = ok ? (KMAJ ? W + (int64_t)m * ldw + k : W + (int64_t)k * ldw + m) : W;
      const float x = *src;
      v[q] = ok ? x : 0.f;
    }
  }
  __device__ __forceinline__ void store(float* __restrict__ dst) const {
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const int idx = threadIdx.x + q * kWG;
      if (idx >= N) break;
      int m, kk;
      if constexpr (KMAJ) { m = idx >> 4; kk = idx & 15; }
      else { kk = idx / (16 * T); m = idx - kk * (16 * T); }
      dst[m * HK_LD + kk] = v[q];
    }
  }
};

// acc[t] += W_chunk(16t + li, 4lk + r) * b[r] for the 4 k-steps r of a chunk,
// t < nt (tiles past nt hold only padding)
template <int T>
__device__ __forceinline__ void chunk_mma(const float* __restrict__ S, const float4 b,
                                          f32x4 (&acc)[T], int nt, int li, int lk) {
#pragma unroll
  for (int t0 = 0; t0 < T; t0 += 4) {
    float4 a[4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (t0 + u < T) a[u] = *reinterpret_cast<const float4*>(S + (16 * (t0 + u) + li) * HK_LD + 4 * lk);
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (t0 + u < T && t0 + u < nt) acc[t0 + u] = mfma4(a[u].x, b.x, acc[t0 + u]);
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (t0 + u < T && t0 + u < nt) acc[t0 + u] = mfma4(a[u].y, b.y, acc[t0 + u]);
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (t0 + u < T && t0 + u < nt) acc[t0 + u] = mfma4(a[u].z, b.z, acc[t0 + u]);
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (t0 + u < T && t0 + u < nt) acc[t0 + u] = mfma4(a[u].w, b.w, acc[t0 + u]);
  }
}

// 4 consecutive features [c, c+4) of a row (zero past n); vec: 16-byte load
__device__ __forceinline__ float4 ld4(const float* __restrict__ p, int c, int n, bool vec) {
  if (vec && c + 3 < n) return *reinterpret_cast<const float4*>(p + c);
  float4 r;
  r.x = c < n ? p[c] : 0.f;
  r.y = c + 1 < n ? p[c + 1] : 0.f;
  r.z = c + 2 < n ? p[c + 2] : 0.f;
  r.w = c + 3 < n ? p[c + 3] : 0.f;
  return r;
}
__device__ __forceinline__ void st4(float* __restrict__ p, int c, int n, bool vec, f32x4 v) {
  if (vec && c + 3 < n) {
    *reinterpret_cast<float4*>(p + c) = float4{v[0], v[1], v[2], v[3]};
    return;
  }
  if (c < n) p[c] = v[0];
  if (c + 1 < n) p[c + 1] = v[1];
  if (c + 2 < n) p[c + 2] = v[2];
  if (c + 3 < n) p[c + 3] = v[3];
}
__device__ __forceinline__ bool al16(const void* p, int64_t ld) {
  return ((reinterpret_cast<uintptr_t>(p) & 15) == 0) && (ld % 4 == 0);
}

// one dense layer over k-blocks held in registers: acc (NT tiles of the
// output) += W(m, k) * in(k) with in's tile c = the previous layer's acc[c]
template <int NT, int KT, bool KMAJ>
__device__ __forceinline__ void layer_from_regs(const float* __restrict__ W, int64_t ldw, int M,
                                                int K, const f32x4 (&in)[KT], f32x4 (&acc)[NT],
                                                float* sW0, float* sW1, int li, int lk) {
  const int nt = (M + 15) >> 4, kt = (K + 15) >> 4;
  Stager<NT, KMAJ> st;
  st.load(W, ldw, M, K, 0);
  st.store(sW0);
  __syncthreads();
  // a runtime loop over the k-blocks (fully unrolled, the three layers'
  // straight-line MFMA code overflowed the instruction cache); `in` is then
  // dynamically indexed and lives in private memory — one 16-byte, cache-
  // resident read per 4*NT MFMAs, fetched a chunk ahead
  f32x4 bc = in[0];
#pragma unroll 1
  for (int c = 0; c < kt; ++c) {
    const bool more = c + 1 < kt;
    f32x4 bn = bc;
    if (more) {
      st.load(W, ldw, M, K, 16 * (c + 1));
      bn = in[c + 1];
    }
    chunk_mma<NT>((c & 1) ? sW1 : sW0, float4{bc[0], bc[1], bc[2], bc[3]}, acc, nt, li, lk);
    if (more) st.store((c & 1) ? sW0 : sW1);
    bc = bn;
    __syncthreads();
  }
}

template <int T1, int T2, int T3>
__global__ void __launch_bounds__(kWG, 2)
head_fwd_fused_kernel(HeadFwdArgs a) {
  if (a.skip && a.skip[0] != 0) return;
  constexpr int TM = T1 > T2 ? (T1 > T3 ? T1 : T3) : (T2 > T3 ? T2 : T3);
  __shared__ __attribute__((aligned(16))) float sW[2][16 * TM * HK_LD];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int li = lane & 15, lk = lane >> 4;
  const int64_t row = (int64_t)blockIdx.x * 64 + wave * 16 + li;
  const bool rok = row < a.rows;
  const int64_t rr = rok ? row : a.rows - 1;
  const float* xr = a.X + rr * a.ldx;
  const bool xvec = al16(a.X, a.ldx);
  // ---- layer 1 over the input (k-blocks of 16 features from global memory)
  f32x4 acc1[T1];
#pragma unroll
  for (int t = 0; t < T1; ++t) acc1[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  {
    const int n1 = (a.h1 + 15) >> 4, kt = (a.K0 + 15) >> 4;
    Stager<T1, true> st;
    st.load(a.W1, a.K0, a.h1, a.K0, 0);
    st.store(sW[0]);
    float4 bx = ld4(xr, 4 * lk, a.K0, xvec);
    __syncthreads();
    for (int c = 0; c < kt; ++c) {
      const bool more = c + 1 < kt;
      float4 bn = bx;
      if (more) {
        st.load(a.W1, a.K0, a.h1, a.K0, 16 * (c + 1));
        bn = ld4(xr, 16 * (c + 1) + 4 * lk, a.K0, xvec);
      }
      chunk_mma<T1>(sW[c & 1], bx, acc1, n1, li, lk);
      if (more) st.store(sW[(c + 1) & 1]);
      bx = bn;
      __syncthreads();
    }
  }
  const bool v1 = al16(a.HA1, a.h1), v2 = al16(a.HA2, a.h2), vy = al16(a.Y, a.ldy);
#pragma unroll
  for (int t = 0; t < T1; ++t) {
    const int m = 16 * t + 4 * lk;
    const float4 bb = ld4(a.b1, m, a.h1, false);
    f32x4 v = acc1[t] + f32x4{bb.x, bb.y, bb.z, bb.w};
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = (v[r] > 0.f && m + r < a.h1) ? v[r] : 0.f;
    acc1[t] = v;
    if (rok && m < a.h1) st4(a.HA1 + row * a.h1, m, a.h1, v1, v);
  }
  // ---- layer 2
  f32x4 acc2[T2];
#pragma unroll
  for (int t = 0; t < T2; ++t) acc2[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  layer_from_regs<T2, T1, true>(a.W2, a.h1, a.h2, a.h1, acc1, acc2, sW[0], sW[1], li, lk);
#pragma unroll
  for (int t = 0; t < T2; ++t) {
    const int m = 16 * t + 4 * lk;
    const float4 bb = ld4(a.b2, m, a.h2, false);
    f32x4 v = acc2[t] + f32x4{bb.x, bb.y, bb.z, bb.w};
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = (v[r] > 0.f && m + r < a.h2) ? v[r] : 0.f;
    acc2[t] = v;
    if (rok && m < a.h2) st4(a.HA2 + row * a.h2, m, a.h2, v2, v);
  }
  // ---- layer 3 (+ bias, tanh for the actor mean)
  f32x4 acc3[T3];
#pragma unroll
  for (int t = 0; t < T3; ++t) acc3[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  layer_from_regs<T3, T2, true>(a.W3, a.h2, a.out, a.h2, acc2, acc3, sW[0], sW[1], li, lk);
#pragma unroll
  for (int t = 0; t < T3; ++t) {
    const int m = 16 * t + 4 * lk;
    if (!rok || m >= a.out) continue;
    const float4 bb = ld4(a.b3, m, a.out, false);
    f32x4 v = acc3[t] + f32x4{bb.x, bb.y, bb.z, bb.w};
    if (a.tanh_out) {
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = tanhf(v[r]);
    }
    st4(a.Y + row * a.ldy, m, a.out, vy, v);
  }
}

template <int T1, int T2, int T3>
__global__ void __launch_bounds__(kWG, 2)
head_bwd_fused_kernel(HeadBwdArgs a) {
  if (a.skip && a.skip[0] != 0) return;
  constexpr int TM = T1 > T2 ? (T1 > T3 ? T1 : T3) : (T2 > T3 ? T2 : T3);
  __shared__ __attribute__((aligned(16))) float sW[2][16 * TM * HK_LD];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int li = lane & 15, lk = lane >> 4;
  const int64_t row = (int64_t)blockIdx.x * 64 + wave * 16 + li;
  const bool rok = row < a.rows;
  const int64_t rr = rok ? row : a.rows - 1;
  // ---- dH2 = (dZ W3) * [HA2 > 0]: one k-block (out <= 16)
  f32x4 acc1[T1];
#pragma unroll
  for (int t = 0; t < T1; ++t) acc1[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  {
    f32x4 dz[1];
    const float4 z = ld4(a.dZ + rr * a.ldz, 4 * lk, a.out, al16(a.dZ, a.ldz));
    dz[0] = f32x4{z.x, z.y, z.z, z.w};
    layer_from_regs<T1, 1, false>(a.W3, a.h2, a.h2, a.out, dz, acc1, sW[0], sW[1], li, lk);
  }
  const bool vm2 = al16(a.HA2, a.h2), vm1 = al16(a.HA1, a.h1);
#pragma unroll
  for (int t = 0; t < T1; ++t) {
    const int m = 16 * t + 4 * lk;
    const float4 mk = ld4(a.HA2 + rr * a.h2, m, a.h2, vm2);
    f32x4 v = acc1[t];
    v[0] = mk.x > 0.f ? v[0] : 0.f; v[1] = mk.y > 0.f ? v[1] : 0.f;
    v[2] = mk.z > 0.f ? v[2] : 0.f; v[3] = mk.w > 0.f ? v[3] : 0.f;
    acc1[t] = v;
    if (rok && m < a.h2) st4(a.dH2 + row * a.h2, m, a.h2, vm2, v);
  }
  // ---- dH1 = (dH2 W2) * [HA1 > 0]:  A(m = j1, k = j2) = W2[j2][j1]
  f32x4 acc2[T2];
#pragma unroll
  for (int t = 0; t < T2; ++t) acc2[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  layer_from_regs<T2, T1, false>(a.W2, a.h1, a.h1, a.h2, acc1, acc2, sW[0], sW[1], li, lk);
#pragma unroll
  for (int t = 0; t < T2; ++t) {
    const int m = 16 * t + 4 * lk;
    const float4 mk = ld4(a.HA1 + rr * a.h1, m, a.h1, vm1);
    f32x4 v = acc2[t];
    v[0] = mk.x > 0.f ? v[0] : 0.f; v[1] = mk.y > 0.f ? v[1] : 0.f;
    v[2] = mk.z > 0.f ? v[2] : 0.f; v[3] = mk.w > 0.f ? v[3] : 0.f;
    acc2[t] = v;
    if (rok && m < a.h1) st4(a.dH1 + row * a.h1, m, a.h1, vm1, v);
  }
  if (a.dxn <= 0) return;
  // ---- dX[:, c] = dH1 W1[:, dx0 + c]:  A(m = c, k = j1) = W1[j1][dx0 + c]
  f32x4 acc3[T3];
#pragma unroll
  for (int t = 0; t < T3; ++t) acc3[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  layer_from_regs<T3, T2, false>(a.W1 + a.dx0, a.in, a.dxn, a.h1, acc2, acc3, sW[0], sW[1], li,
                                 lk);
  if (!rok) return;
  const bool vx = al16(a.dX, a.lddx);
  const bool vmk = a.mask && al16(a.mask, a.ldm);
#pragma unroll
  for (int t = 0; t < T3; ++t) {
    const int m = 16 * t + 4 * lk;
    if (m >= a.dxn) continue;
    f32x4 v = acc3[t];
    if (a.mask) {
      const float4 mk = ld4(a.mask + row * a.ldm, m, a.dxn, vmk);
      v[0] = mk.x > 0.f ? v[0] : 0.f; v[1] = mk.y > 0.f ? v[1] : 0.f;
      v[2] = mk.z > 0.f ? v[2] : 0.f; v[3] = mk.w > 0.f ? v[3] : 0.f;
    }
    st4(a.dX + row * a.lddx, m, a.dxn, vx, v);
  }
}

// tile capacities of the compiled variants: h1 <= 304, h2 <= 208, out <= 16,
// input-gradient columns <= 112 (PPO heads 300x200 and smaller over the LSTM's 100
// outputs; wider inputs, e.g. the pixel MLP's 256 CNN features, take the layer GEMMs)
constexpr int HF_T1 = 19, HF_T2 = 13, HF_T3 = 1;
constexpr int HB_T1 = 13, HB_T2 = 19, HB_T3 = 7;

static int use_head_fused() {
  static int u = -1;
  if (u < 0) {
    const char* e = getenv("SMI_HEAD_FUSED");
    u = (e && e[0] == '0') ? 0 : 1;
  }
  return u;
}

int launch_head_fwd_fused(const float* X, int64_t ldx, int K0, const float* P, int h1, int h2,
                          int out, int64_t oW1, int64_t ob1, int64_t oW2, int64_t ob2,
                          int64_t oW3, int64_t ob3, int tanh_out, float* HA1, float* HA2,
                          float* Y, int64_t ldy, int64_t rows, hipStream_t st, const int* skip) {
  if (!use_head_fused() || h1 > 16 * HF_T1 || h2 > 16 * HF_T2 || out > 16 * HF_T3 || K0 < 1 ||
      h1 < 1 || h2 < 1 || out < 1)
    return SMI_E_NOFIT;
  if (rows <= 0) return SMI_OK;
  HeadFwdArgs a{X, ldx, K0, P + oW1, P + ob1, P + oW2, P + ob2, P + oW3, P + ob3, h1, h2, out,
                tanh_out, HA1, HA2, Y, ldy, rows, skip};
  const int kslot = ktime_begin(st);
  hipLaunchKernelGGL((head_fwd_fused_kernel<HF_T1, HF_T2, HF_T3>), dim3((unsigned)((rows + 63) / 64)),
                     dim3(kWG), 0, st, a);
  ktime_end(kslot, KT_GEMM_FWD, 2.0 * (double)rows * ((double)K0 * h1 + (double)h1 * h2 + (double)h2 * out),
            st);
  return check_launch("head_fwd_fused_kernel");
}

int launch_head_bwd_fused(const float* dZ, int64_t ldz, int out, const float* P, int in, int h1,
                          int h2, int64_t oW1, int64_t oW2, int64_t oW3, const float* HA1,
                          const float* HA2, float* dH2, float* dH1, float* dX, int64_t lddx,
                          int dx0, int dxn, const float* mask, int64_t ldm, int64_t rows,
                          hipStream_t st, const int* skip) {
  if (!use_head_fused() || h2 > 16 * HB_T1 || h1 > 16 * HB_T2 || dxn > 16 * HB_T3 || out > 16 ||
      out < 1 || h1 < 1 || h2 < 1 || dx0 < 0 || dx0 + dxn > in)
    return SMI_E_NOFIT;
  if (rows <= 0) return SMI_OK;
  HeadBwdArgs a{dZ, ldz, out, P + oW1, in, P + oW2, P + oW3, h1, h2, HA1, HA2, dH2, dH1,
                dX, lddx, dx0, dxn, mask, ldm, rows, skip};
  const int kslot = ktime_begin(st);
  hipLaunchKernelGGL((head_bwd_fused_kernel<HB_T1, HB_T2, HB_T3>), dim3((unsigned)((rows + 63) / 64)),
                     dim3(kWG), 0, st, a);
  ktime_end(kslot, KT_GEMM_DX,
            2.0 * (double)rows * ((double)out * h2 + (double)h2 * h1 + (double)h1 * (dxn > 0 ? dxn : 0)),
            st);
  return check_launch("head_bwd_fused_kernel");
}

}  // namespace smi
