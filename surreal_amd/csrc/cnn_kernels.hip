// cnn_kernels.hip — the pixel stem of PPOModel: CNNStemNetwork
// (surreal/model/model_builders/builders.py:8-33) applied to obs/255
// (ppo_net.py:268-273,368-375):
//   conv 8x8 stride 4 (C -> 16) -> ReLU -> conv 4x4 stride 2 (16 -> 32) -> ReLU
//   -> Flatten (C,H,W order) -> Linear(F) -> ReLU
//
// The two convolutions of one image run in one workgroup as implicit GEMMs on
// v_mfma_f32_16x16x4_f32: the uint8 image (21 KB for 3x84x84) and the conv-1
// activation (25.6 KB) stay in LDS, the weights live in registers as MFMA B
// operands, and only A1 (kept for the backward) and A2 leave the CU.  The
// Linear layer is a plain GEMM on the split-K MFMA engine (linear_kernels.hip).
//
// Backward: Linear dW/dX on the GEMM engine, then one workgroup per image
// computes, from LDS, the conv-2 weight gradient, the conv-2 input gradient
// (a transposed convolution, split into the four stride-parity classes so
// every tap is dense) masked by ReLU, and the conv-1 weight gradient.  Weight
// gradients accumulate in registers across the images of a workgroup and are
// summed over workgroups by the fixed-order slab reducer: deterministic.
//
// Pixel scaling: torch computes conv(fl(u / 255)).  The kernels feed the raw
// byte values (exact in fp32) to the MFMAs and divide the conv-1 sums by 255
// (IEEE division) in the epilogue — one v_cvt per operand instead of a
// correctly rounded division.  Same result up to fp32 rounding of the sum
// (the parity bar); a one-hot filter gives exactly fl(u / 255)
// (test_u8_scaling_bit_exact).
#include "smi_device.hpp"
#include "smi_internal.hpp"

namespace smi {

int launch_slab_reduce(const float* part, int S, int64_t n, float* out, hipStream_t st,
                       const int* skip);

__device__ __forceinline__ float u8f(unsigned u, int byte) {
  return (float)((u >> (8 * byte)) & 0xffu);
}

__device__ __forceinline__ const unsigned char* pix_of(const PixRows& pr, int64_t n) {
  const int64_t t = n / pr.B, b = n - t * pr.B;
  return t < pr.T ? pr.pix + (b * pr.T + t) * pr.img_bytes : pr.pix_next + b * pr.img_bytes;
}

__host__ __device__ inline int64_t lds_img_bytes(const CnnGeom& g) { return (g.img + 15) & ~(int64_t)15; }

// ------------------------------------------------------------------ forward
// One workgroup (4 waves) per image, grid-stride over images.
//   conv1: implicit GEMM M = P1 pixels, N = 16 channels, K = 64*C; wave w owns
//          pixel tiles w, w+4, ...; the K order is permuted so one lane reads
//          8 consecutive bytes (kx = 0..7 of one (ci, ky) image row) per 8 MFMAs.
//   conv2: M = P2 pixels, N = 32, K = 256; wave w owns channel tile w>>1 and
//          pixel tiles (w&1), (w&1)+2, ...; one lane reads 4 consecutive A1
//          floats (kx = 0..3) per 4 MFMAs.
// RGB (C = 3): 3 waves per SIMD (168 VGPRs, a few bytes of scratch) beat 2
// waves at 176: 132 vs 143 us per 2688-image forward (tools/bench_cnn.py).
// Three stacked RGB frames (C = 9, DDPG's frame_stacks = 3, ddpg_configs.py:
// 114): the 144 conv-1 weight registers need one wave per SIMD.
// per-thread 16-byte chunk counts of an 84 x 84 frame's staging (image, A1,
// dA2), register arrays of the forward's batched image loads and the
// backward's next-image prefetch (larger frames: a tail loop / PF off)
#ifndef SMI_CNN_FWD_KB
#define SMI_CNN_FWD_KB 6
#endif
template <int C> struct CnnPf {
  static constexpr int KI = C <= 3 ? 6 : 16;     // uint4 of the uint8 image
  static constexpr int KA = 7;                   // float4 of A1 (16 x P1)
  static constexpr int KD = 3;                   // float4 of dA2 (flat)
};

template <int C>
__global__ void __launch_bounds__(kWG) __attribute__((amdgpu_waves_per_eu(C <= 3 ? 3 : 1, C <= 3 ? 3 : 1)))
cnn_fwd_kernel(const float* __restrict__ prm, PixRows pr, int H, int W, int64_t rows,
               float* __restrict__ A1g, float* __restrict__ A2g, const int* skip) {
  if (skip && skip[0] != 0) return;
  const CnnGeom g = cnn_geom(C, H, W, 1);
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned char* img = smem;
  float* a1 = reinterpret_cast<float*>(smem + lds_img_bytes(g));
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, lg = l >> 4, lm = l & 15;

  float w1r[16 * C];
#pragma unroll
  for (int j = 0; j < 16 * C; ++j) {
    const int r = (j >> 3) * 4 + lg;                 // image row index ci*8 + ky
    w1r[j] = prm[g.oW1 + (int64_t)lm * g.K1 + r * 8 + (j & 7)];
  }
  const int ct = w >> 1;
  float w2r[64];
#pragma unroll
  for (int j = 0; j < 64; ++j) {
    const int r = (j >> 2) * 4 + lg;                 // ci*4 + ky
    w2r[j] = prm[g.oW2 + (int64_t)(ct * 16 + lm) * 256 + r * 4 + (j & 3)];
  }
  const float b1 = prm[g.ob1 + lm], b2 = prm[g.ob2 + ct * 16 + lm];
  const int nt1 = (g.P1 + 15) >> 4, nt2 = (g.P2 + 15) >> 4;
  const int HW = H * W;

  for (int64_t n = blockIdx.x; n < rows; n += gridDim.x) {
    {   // all of a thread's image loads first, then its LDS stores: one
        // memory round trip per image instead of one per 16-byte chunk
      typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
      // (batches of KB chunks: the RGB kernel's 3-waves/SIMD register budget
      // spills weights with more staging registers live)
      constexpr int KB = SMI_CNN_FWD_KB;
      const u32x4* src = reinterpret_cast<const u32x4*>(pix_of(pr, n));
      u32x4* dst = reinterpret_cast<u32x4*>(img);
      const int nv = (int)(g.img >> 4);
      for (int i0 = tid; i0 < nv; i0 += KB * kWG) {
        u32x4 v[KB];
#pragma unroll
        for (int k = 0; k < KB; ++k) v[k] = src[min(i0 + k * kWG, nv - 1)];
#pragma unroll
        for (int k = 0; k < KB; ++k)
          if (i0 + k * kWG < nv) dst[i0 + k * kWG] = v[k];
      }
    }
    __syncthreads();
    // ---- conv 1: two pixel tiles (two independent MFMA chains) per pass
    for (int pt = w; pt < nt1; pt += 8) {
      const int ptb = pt + 4 < nt1 ? pt + 4 : pt;      // second tile (dup when odd)
      int pa = pt * 16 + lm, pb2 = ptb * 16 + lm;
      pa = pa < g.P1 ? pa : g.P1 - 1;
      pb2 = pb2 < g.P1 ? pb2 : g.P1 - 1;
      const int oya = pa / g.W1, oxa = pa - oya * g.W1;
      const int oyb = pb2 / g.W1, oxb = pb2 - oyb * g.W1;
      const unsigned char* basea = img + oya * 4 * W + oxa * 4;
      const unsigned char* baseb = img + oyb * 4 * W + oxb * 4;
      f32x4 acc = {0.f, 0.f, 0.f, 0.f}, acc2 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int rb = 0; rb < 2 * C; ++rb) {
        const int r = rb * 4 + lg;
        const int ro = (r >> 3) * HW + (r & 7) * W;
        const unsigned* qa = reinterpret_cast<const unsigned*>(basea + ro);
        const unsigned* qb = reinterpret_cast<const unsigned*>(baseb + ro);
        const unsigned a0 = qa[0], a1w = qa[1], b0 = qb[0], b1w = qb[1];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          acc = mfma4(u8f(a0, u), w1r[rb * 8 + u], acc);
          acc2 = mfma4(u8f(b0, u), w1r[rb * 8 + u], acc2);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          acc = mfma4(u8f(a1w, u), w1r[rb * 8 + 4 + u], acc);
          acc2 = mfma4(u8f(b1w, u), w1r[rb * 8 + 4 + u], acc2);
        }
      }
      // D[pixel tile*16 + lg*4 + i][channel lm]; P1 % 4 == 0 (checked on the host)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        if (h == 1 && ptb == pt) break;
        const f32x4 s4 = h == 0 ? acc : acc2;
        const int p0 = (h == 0 ? pt : ptb) * 16 + lg * 4;
        if (p0 < g.P1) {
          float4 v;
          v.x = fmaxf(s4[0] / 255.0f + b1, 0.f); v.y = fmaxf(s4[1] / 255.0f + b1, 0.f);
          v.z = fmaxf(s4[2] / 255.0f + b1, 0.f); v.w = fmaxf(s4[3] / 255.0f + b1, 0.f);
          *reinterpret_cast<float4*>(a1 + lm * g.P1 + p0) = v;
          if (A1g) *reinterpret_cast<float4*>(A1g + n * (int64_t)(16 * g.P1) + lm * g.P1 + p0) = v;
        }
      }
    }
    __syncthreads();
    // ---- conv 2
    for (int pt = (w & 1); pt < nt2; pt += 2) {
      int p = pt * 16 + lm;
      p = p < g.P2 ? p : g.P2 - 1;
      const int oy = p / g.W2, ox = p - oy * g.W2;
      const float* base = a1 + oy * 2 * g.W1 + ox * 2;
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int rb = 0; rb < 16; ++rb) {
        const int r = rb * 4 + lg;
        const float* q = base + (r >> 2) * g.P1 + (r & 3) * g.W1;
        const float2 x0 = *reinterpret_cast<const float2*>(q);
        const float2 x1 = *reinterpret_cast<const float2*>(q + 2);
        acc = mfma4(x0.x, w2r[rb * 4 + 0], acc);
        acc = mfma4(x0.y, w2r[rb * 4 + 1], acc);
        acc = mfma4(x1.x, w2r[rb * 4 + 2], acc);
        acc = mfma4(x1.y, w2r[rb * 4 + 3], acc);
      }
      float* dst = A2g + n * (int64_t)g.flat + (ct * 16 + lm) * g.P2;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int pp = pt * 16 + lg * 4 + i;
        if (pp < g.P2) dst[pp] = fmaxf(acc[i] + b2, 0.f);
      }
    }
    // the next image's staging only overwrites img (read before the barrier
    // above); its conv-1 writes a1 after the next barrier
  }
}

// ----------------------------------------------------------------- backward
// One workgroup per image slot (grid-stride); partial weight gradients of the
// workgroup go to part[blockIdx.x][0 .. g.nconv) in the flat layout
// [W1 | b1 | W2 | b2].
//   (b) dW2[co][k] += sum_p dA2[co][p] * col(A1)[p][k]   M=32 N=256 K=P2
//   (c) dA1 = relu'(A1) * convT(dA2, W2): wave w handles the positions with
//       (y % 2, x % 2) = (w >> 1, w & 1); its taps ky = py + {0,2},
//       kx = px + {0,2} are all dense: M = positions, N = 16, K = 32 x 4 taps
//   (d) dW1[co][k] += sum_p dA1[co][p] * col(img/255)[p][k]  M=16 N=64C K=P1
// Next-image prefetch (PF): the image, A1 and dA2 of the workgroup's next
// image are loaded into registers (clamped addresses, unconditional loads)
// right after this image's staging barrier and written to LDS at the top of
// the next iteration, so their latency hides behind this image's three MFMA
// passes instead of ~14 serialized load -> LDS-store round trips per image.
// Per-thread register counts for 84 x 84 frames (host-checked, else PF off).

template <int C, bool PF>
__global__ void __launch_bounds__(kWG) __attribute__((amdgpu_waves_per_eu(1, PF ? 2 : 4)))
cnn_bwd_kernel(const float* __restrict__ prm, PixRows pr, int H, int W, int64_t rows,
               const float* __restrict__ A1g, const float* __restrict__ dA2g,
               float* __restrict__ part, const int* skip) {
  if (skip && skip[0] != 0) return;
  const CnnGeom g = cnn_geom(C, H, W, 1);
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned char* img = smem;
  float* a1 = reinterpret_cast<float*>(smem + lds_img_bytes(g));       // A1, then dA1
  float* da2 = a1 + 16 * g.P1;
  float* red = da2 + round4(g.flat);
  int* ofs1 = reinterpret_cast<int*>(red + kWG);       // conv-1 pixel p -> byte offset
  int* ofs2 = ofs1 + g.P1;                              // conv-2 pixel p -> A1 offset
  for (int p = threadIdx.x; p < g.P1; p += kWG) {
    const int oy = p / g.W1;
    ofs1[p] = oy * 4 * W + (p - oy * g.W1) * 4;
  }
  for (int p = threadIdx.x; p < g.P2; p += kWG) {
    const int oy = p / g.W2;
    ofs2[p] = oy * 2 * g.W1 + (p - oy * g.W2) * 2;
  }
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, lg = l >> 4, lm = l & 15;
  const int HW = H * W;

  // (b) roles
  const int ct = w >> 1, kt0 = (w & 1) * 8;
  int koff2[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    const int k = (kt0 + t) * 16 + lm;               // ci*16 + ky*4 + kx
    koff2[t] = (k >> 4) * g.P1 + ((k >> 2) & 3) * g.W1 + (k & 3);
  }
  f32x4 acc2[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) acc2[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  // (c) roles
  const int py = w >> 1, px = w & 1;
  const int NY = (g.H1 - py + 1) >> 1, NX = (g.W1 - px + 1) >> 1, Q = NY * NX;
  const int ty = lg >> 1, tx = lg & 1;
  float w2c[32];
#pragma unroll
  for (int j = 0; j < 32; ++j)
    w2c[j] = prm[g.oW2 + (int64_t)j * 256 + lm * 16 + (py + 2 * ty) * 4 + (px + 2 * tx)];
  // (d) roles: k tiles w*C .. w*C + C-1 (4C tiles of 16 over 64C columns)
  int koff1[C];
#pragma unroll
  for (int t = 0; t < C; ++t) {
    const int k = (w * C + t) * 16 + lm;             // ci*64 + ky*8 + kx
    koff1[t] = (k >> 6) * HW + ((k >> 3) & 7) * W + (k & 7);
  }
  f32x4 acc1[C];
#pragma unroll
  for (int t = 0; t < C; ++t) acc1[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  float db2p = 0.f, db1p = 0.f;

  const int nvi = (int)(g.img >> 4), nva = 4 * g.P1, nvd = g.flat >> 2;
  constexpr int KI = PF ? CnnPf<C>::KI : 1, KA = PF ? CnnPf<C>::KA : 1, KD = PF ? CnnPf<C>::KD : 1;
  // ext-vector element types (the HIP vector structs kept these arrays in
  // scratch: SROA does not split them)
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  u32x4 pfi[KI];
  f32x4 pfa[KA], pfd[KD];
#define SMI_CNN_FETCH(n_)                                                                   \
  do {                                                                                      \
    const int64_t nn_ = (n_);                                                               \
    const u32x4* si_ = reinterpret_cast<const u32x4*>(pix_of(pr, nn_));                     \
    const f32x4* s1_ = reinterpret_cast<const f32x4*>(A1g + nn_ * (int64_t)(16 * g.P1));    \
    const f32x4* s2_ = reinterpret_cast<const f32x4*>(dA2g + nn_ * (int64_t)g.flat);        \
    _Pragma("unroll") for (int k = 0; k < KI; ++k) pfi[k] = si_[min(tid + k * kWG, nvi - 1)]; \
    _Pragma("unroll") for (int k = 0; k < KA; ++k) pfa[k] = s1_[min(tid + k * kWG, nva - 1)]; \
    _Pragma("unroll") for (int k = 0; k < KD; ++k) pfd[k] = s2_[min(tid + k * kWG, nvd - 1)]; \
  } while (0)
  if (PF && (int64_t)blockIdx.x < rows) SMI_CNN_FETCH(blockIdx.x);
  for (int64_t n = blockIdx.x; n < rows; n += gridDim.x) {
    if constexpr (PF) {
      u32x4* dst = reinterpret_cast<u32x4*>(img);
      f32x4* d1 = reinterpret_cast<f32x4*>(a1);
      f32x4* d2 = reinterpret_cast<f32x4*>(da2);
#pragma unroll
      for (int k = 0; k < KI; ++k) if (tid + k * kWG < nvi) dst[tid + k * kWG] = pfi[k];
#pragma unroll
      for (int k = 0; k < KA; ++k) if (tid + k * kWG < nva) d1[tid + k * kWG] = pfa[k];
#pragma unroll
      for (int k = 0; k < KD; ++k) if (tid + k * kWG < nvd) d2[tid + k * kWG] = pfd[k];
    } else {
      const uint4* src = reinterpret_cast<const uint4*>(pix_of(pr, n));
      uint4* dst = reinterpret_cast<uint4*>(img);
      for (int i = tid; i < nvi; i += kWG) dst[i] = src[i];
      const float4* s1 = reinterpret_cast<const float4*>(A1g + n * (int64_t)(16 * g.P1));
      float4* d1 = reinterpret_cast<float4*>(a1);
      for (int i = tid; i < nva; i += kWG) d1[i] = s1[i];
      const float4* s2 = reinterpret_cast<const float4*>(dA2g + n * (int64_t)g.flat);
      float4* d2 = reinterpret_cast<float4*>(da2);
      for (int i = tid; i < nvd; i += kWG) d2[i] = s2[i];
    }
    __syncthreads();
    if (PF && n + gridDim.x < rows) SMI_CNN_FETCH(n + gridDim.x);
    // ---- (b) conv-2 weight gradient
    for (int j = 0; j < (g.P2 + 3) >> 2; ++j) {
      const int p = 4 * j + lg;
      const bool ok = p < g.P2;
      const int pc = ok ? p : g.P2 - 1;
      const int pb = ofs2[pc];
      const float av = da2[(ct * 16 + lm) * g.P2 + pc];
      const float a = ok ? av : 0.f;
#pragma unroll
      for (int t = 0; t < 8; ++t) acc2[t] = mfma4(a, a1[koff2[t] + pb], acc2[t]);
    }
    {
      const int ch = tid >> 3;
      for (int p = tid & 7; p < g.P2; p += 8) db2p += da2[ch * g.P2 + p];
    }
    __syncthreads();
    // ---- (c) conv-2 input gradient, in place over A1 (ReLU mask from A1);
    // two position tiles per pass (two independent MFMA chains)
    for (int qt = 0; qt < (Q + 15) >> 4; qt += 2) {
      int off[2];
      bool okq[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int q = (qt + h) * 16 + lm;
        const int qc = q < Q ? q : Q - 1;
        const int yy = qc / NX, xx = qc - yy * NX;
        const int oy = yy - ty, ox = xx - tx;
        okq[h] = q < Q && oy >= 0 && oy < g.H2 && ox >= 0 && ox < g.W2;
        off[h] = okq[h] ? oy * g.W2 + ox : 0;
      }
      f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1c = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int j = 0; j < 32; ++j) {
        const float v0 = da2[j * g.P2 + off[0]];
        const float v1 = da2[j * g.P2 + off[1]];
        acc0 = mfma4(okq[0] ? v0 : 0.f, w2c[j], acc0);
        acc1c = mfma4(okq[1] ? v1 : 0.f, w2c[j], acc1c);
      }
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const f32x4 s4 = h == 0 ? acc0 : acc1c;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int qq = (qt + h) * 16 + lg * 4 + i;
          if (qq < Q) {
            const int y2 = qq / NX, x2 = qq - y2 * NX;
            const int idx = lm * g.P1 + (2 * y2 + py) * g.W1 + (2 * x2 + px);
            a1[idx] = a1[idx] > 0.f ? s4[i] : 0.f;
          }
        }
      }
    }
    __syncthreads();
    // ---- (d) conv-1 weight gradient
    for (int j = 0; j < (g.P1 + 3) >> 2; ++j) {
      const int p = 4 * j + lg;
      const bool ok = p < g.P1;
      const int pc = ok ? p : g.P1 - 1;
      const int pb = ofs1[pc];
      const float av = a1[lm * g.P1 + pc];
      const float a = ok ? av : 0.f;
#pragma unroll
      for (int t = 0; t < C; ++t)           // raw bytes; / 255 when the partial is written
        acc1[t] = mfma4(a, (float)img[koff1[t] + pb], acc1[t]);
    }
    {
      const int ch = tid >> 4;
      for (int p = tid & 15; p < g.P1; p += 16) db1p += a1[ch * g.P1 + p];
    }
    __syncthreads();
  }

  // ---- partials: [W1 | b1 | W2 | b2] of this workgroup
  float* out = part + (int64_t)blockIdx.x * g.nconv;
#pragma unroll
  for (int t = 0; t < 8; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int co = ct * 16 + lg * 4 + i, k = (kt0 + t) * 16 + lm;
      out[g.oW2 + co * 256 + k] = acc2[t][i];
    }
#pragma unroll
  for (int t = 0; t < C; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int co = lg * 4 + i, k = (w * C + t) * 16 + lm;
      out[g.oW1 + co * g.K1 + k] = acc1[t][i] / 255.0f;
    }
  red[tid] = db2p;
  __syncthreads();
  if (tid < 32) {
    float s = 0.f;
    for (int u = 0; u < 8; ++u) s += red[tid * 8 + u];
    out[g.ob2 + tid] = s;
  }
  __syncthreads();
  red[tid] = db1p;
  __syncthreads();
  if (tid < 16) {
    float s = 0.f;
    for (int u = 0; u < 16; ++u) s += red[tid * 16 + u];
    out[g.ob1 + tid] = s;
  }
}
#undef SMI_CNN_FETCH

// ------------------------------------------------------------------- host
static int cnn_check(const CnnGeom& g) {
  if (g.C != 3 && g.C != 9)
    return set_error(SMI_E_ARG, "cnn: 3 (one RGB frame) or 9 (three stacked RGB frames) channels");
  if (g.H1 < 4 || g.W1 < 4 || g.H2 < 1 || g.W2 < 1)
    return set_error(SMI_E_ARG, "cnn: image smaller than the two convolutions");
  if ((g.P2 + 15) / 16 > 6)
    return set_error(SMI_E_ARG, "cnn: conv-2 output larger than 96 pixels (84x84 gives 81)");
  if (g.W % 4 != 0 || g.img % 16 != 0 || g.P1 % 4 != 0 || g.W1 % 2 != 0 || g.flat % 4 != 0)
    return set_error(SMI_E_ARG, "cnn: need W % 4 == 0, C*H*W % 16 == 0, even conv-1 width, "
                                "conv-1 pixels % 4 == 0 (84x84 qualifies)");
  if (g.F < 1) return set_error(SMI_E_ARG, "cnn: feature dim must be >= 1");
  return SMI_OK;
}

static size_t cnn_fwd_lds(const CnnGeom& g) { return (size_t)lds_img_bytes(g) + (size_t)64 * g.P1; }
static size_t cnn_bwd_lds(const CnnGeom& g) {
  return (size_t)lds_img_bytes(g) + (size_t)64 * g.P1 + 4 * (size_t)round4(g.flat) + 4 * kWG +
         4 * (size_t)(g.P1 + g.P2);
}

int cnn_bwd_grid(int64_t rows) { return (int)(rows < kCnnPartials ? rows : kCnnPartials); }

int cnn_forward(const float* prm, const PixRows& pr, int C, int H, int W, int F, int64_t rows,
                float* A1, float* A2, float* feat, int64_t ldf, hipStream_t st, const int* skip) {
  const CnnGeom g = cnn_geom(C, H, W, F);
  RC_CHECK(cnn_check(g));
  if (rows < 1) return SMI_OK;
  if ((reinterpret_cast<uintptr_t>(pr.pix) | reinterpret_cast<uintptr_t>(pr.pix_next)) & 15)
    return set_error(SMI_E_ARG, "cnn: pixel buffers must be 16-byte aligned");
  const size_t lds = cnn_fwd_lds(g);
  auto k = C == 9 ? cnn_fwd_kernel<9> : cnn_fwd_kernel<3>;
  allow_lds(k, lds);
  const int64_t rg = resident_grid(k, kWG, lds);
  const int grid = (int)(rows < rg ? rows : rg);
  const int kt = ktime_begin(st);
  hipLaunchKernelGGL(k, dim3(grid), dim3(kWG), lds, st, prm, pr, H, W, rows, A1, A2, skip);
  ktime_end(kt, KT_CNN_FWD, 2.0 * (double)rows * (16.0 * g.P1 * g.K1 + 32.0 * g.P2 * 256.0), st);
  RC_CHECK(check_launch("cnn_fwd_kernel"));
  return launch_linear_fwd(A2, g.flat, (int)rows, g.flat, prm + g.oWf, g.flat, prm + g.obf, F,
                           ACT_RELU, feat, ldf, st, skip);
}

int cnn_backward(const float* prm, const PixRows& pr, int C, int H, int W, int F, int64_t rows,
                 const float* A1, const float* A2, const float* dz, int64_t lddz, float* grad,
                 float* dA2, float* part, hipStream_t st, const int* skip) {
  const CnnGeom g = cnn_geom(C, H, W, F);
  RC_CHECK(cnn_check(g));
  if (rows < 1) return SMI_OK;
  RC_CHECK(launch_linear_bwd_dw(dz, lddz, (int)rows, F, A2, g.flat, g.flat, grad + g.oWf, g.flat,
                                grad + g.obf, 0, st, skip));
  RC_CHECK(launch_linear_bwd_dx(dz, lddz, (int)rows, F, prm + g.oWf, g.flat, g.flat, A2, g.flat,
                                dA2, g.flat, st, skip));
  const size_t lds = cnn_bwd_lds(g);
  // next-image prefetch when the frame fits its register arrays (84 x 84 does)
  static const bool pf_on = [] { const char* e = getenv("SMI_CNN_PF"); return !(e && e[0] == '0'); }();
  auto fits = [&](auto pf) {
    using P = decltype(pf);
    return (g.img >> 4) <= (int64_t)P::KI * kWG && 4 * g.P1 <= P::KA * kWG && (g.flat >> 2) <= P::KD * kWG;
  };
  const bool pf = pf_on && (C == 9 ? fits(CnnPf<9>{}) : fits(CnnPf<3>{}));
  auto k = C == 9 ? (pf ? cnn_bwd_kernel<9, true> : cnn_bwd_kernel<9, false>)
                  : (pf ? cnn_bwd_kernel<3, true> : cnn_bwd_kernel<3, false>);
  allow_lds(k, lds);
  const int grid = cnn_bwd_grid(rows);
  const int kt = ktime_begin(st);
  hipLaunchKernelGGL(k, dim3(grid), dim3(kWG), lds, st, prm, pr, H, W, rows, A1, dA2, part, skip);
  ktime_end(kt, KT_CNN_BWD,
            2.0 * (double)rows * (32.0 * g.P2 * 256.0 * 2.0 + 16.0 * g.P1 * g.K1), st);
  RC_CHECK(check_launch("cnn_bwd_kernel"));
  return launch_slab_reduce(part, grid, g.nconv, grad, st, skip);
}

}  // namespace smi
