// ppo_gae.hip — PPO learner GAE/returns on gfx950.
//
//   critic_gae_kernel      PPOLearner._gae_and_return, non-RNN (ppo.py:355-418):
//                          critic MLP over cat(obs, obs_next) + window sums
//   gae_windows_kernel     windowed GAE given values (ppo.py:387-406), streaming
//
// Numerics follow the reference's fp32 op order where it is observable
// (see DESIGN.md §Numerics).
#include "smi_device.hpp"
#include "smi_internal.hpp"
namespace smi {

// ============================================================ critic + GAE
// One workgroup loops over chunks of CS whole segments (grid-stride).  The
// chunk's rows (b, t), t in [0, T] (t == T is obs_next) are flattened and run
// through the critic MLP in 64-row tiles; values stay in LDS, then one thread
// per segment forms the window sums.
struct CriticGaeArgs {
  const float* params; int D, H1, H2;
  int use_zf; const float *zf_sum, *zf_sumsq, *zf_count; float zf_eps;
  const float *obs, *obs_next, *rewards, *dones;
  int B, T, CS;
  const float *gtab, *ltab; float gamma, gamma_T;
  float *values, *adv, *ret;
  int params_in_lds;
};

__global__ void __launch_bounds__(kWG)
critic_gae_kernel(CriticGaeArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const MlpLayout L = mlp_layout(a.D, a.H1, a.H2, 1, 0);
  const int ldX = pad_ld(a.D), ldH1 = pad_ld(a.H1), ldH2 = pad_ld(a.H2), ldO = pad_small(1);
  const int T1 = a.T + 1;
  // LDS carve (floats)
  float* zmean = sm;                       // [D]
  float* zstd = zmean + round4(a.D);       // [D]
  float* X0 = zstd + round4(a.D);          // [64][ldX]
  float* H1 = X0 + kRT * ldX;              // [64][ldH1]
  float* H2 = H1 + kRT * ldH1;             // [64][ldH2]
  float* OUT = H2 + kRT * ldH2;            // [64][ldO]
  float* vals = OUT + kRT * ldO;           // [CS*T1]
  float* P = vals + round4(a.CS * T1);     // padded params (if in LDS)

  if (a.use_zf) zfilter_colstats(a.zf_sum, a.zf_sumsq, a.zf_count, a.zf_eps, a.D, zmean, zstd);
  MlpView V;
  if (a.params_in_lds) {
    mlp_load_lds(L, a.params, P);
    V = view_padded(L, P);
  } else {
    V = view_flat(L, a.params);
  }
  // zero H/OUT padding columns once (finite values only are ever written)
  for (int e = threadIdx.x; e < kRT * (ldH1 + ldH2 + ldO); e += kWG) H1[e] = 0.f;
  __syncthreads();

  const int nchunks = (a.B + a.CS - 1) / a.CS;
  for (int ch = blockIdx.x; ch < nchunks; ch += gridDim.x) {
    const int b0 = ch * a.CS;
    const int nseg = min(a.CS, a.B - b0);
    const int rows = nseg * T1;
    for (int r0 = 0; r0 < rows; r0 += kRT) {
      // gather rows (b, t) -> X0 with the ZFilter fused
      for (int e = threadIdx.x; e < kRT * ldX; e += kWG) {
        const int r = e / ldX, c = e - r * ldX;
        const int q = r0 + r;
        float v = 0.f;
        if (q < rows && c < a.D) {
          const int sb = q / T1, t = q - sb * T1;
          const int64_t b = b0 + sb;
          v = (t < a.T) ? a.obs[(b * a.T + t) * a.D + c] : a.obs_next[b * a.D + c];
          if (a.use_zf) {
            v = (v - zmean[c]) / zstd[c];
            v = fminf(fmaxf(v, -5.f), 5.f);
          }
        }
        X0[e] = v;
      }
      __syncthreads();
      dense_fwd<ACT_RELU>(X0, ldX, V.W1, V.ld1, V.b1, a.D, a.H1, H1, ldH1);
      __syncthreads();
      dense_fwd<ACT_RELU>(H1, ldH1, V.W2, V.ld2, V.b2, a.H1, a.H2, H2, ldH2);
      __syncthreads();
      dense_fwd<ACT_NONE>(H2, ldH2, V.W3, V.ld3, V.b3, a.H2, 1, OUT, ldO);
      __syncthreads();
      for (int r = threadIdx.x; r < kRT; r += kWG)
        if (r0 + r < rows) vals[r0 + r] = OUT[r * ldO];
      __syncthreads();
    }
    // values[:, 1:] *= 1 - dones   (ppo.py:387)
    for (int q = threadIdx.x; q < rows; q += kWG) {
      const int sb = q / T1, t = q - sb * T1;
      if (t > 0) {
        const int64_t b = b0 + sb;
        vals[q] = vals[q] * (1.f - a.dones[b * a.T + t - 1]);
      }
      if (a.values) a.values[(int64_t)b0 * T1 + q] = vals[q];
    }
    __syncthreads();
    // window sums (ppo.py:409-411), one thread per segment
    for (int sb = threadIdx.x; sb < nseg; sb += kWG) {
      const int64_t b = b0 + sb;
      const float* r = a.rewards + b * a.T;
      const float* v = vals + sb * T1;
      float sr = 0.f, sa = 0.f;
      for (int t = 0; t < a.T; ++t) {
        sr += a.gtab[t] * r[t];
        const float td = (r[t] + a.gamma * v[t + 1]) - v[t];
        sa += (td * a.gtab[t]) * a.ltab[t];
      }
      a.ret[b] = sr + v[a.T] * a.gamma_T;
      a.adv[b] = sa;
    }
    __syncthreads();
  }
}

// ===================================================== streaming GAE windows
// values [B][T+1], rewards/dones [B][T] -> adv/ret [B][E]  (ppo.py:387-406).
// HBM-bound.  A workgroup stages a contiguous block of SB segments of r, d, V
// through LDS with 16-byte coalesced loads (the three arrays are contiguous per
// segment block; SB is a multiple of 4, so every block starts 16-byte aligned).
//   pass 1 (row-mapped: TPR = 2^k >= T threads per segment row, no divides):
//          td[s][t] = r + gamma * V[t+1](1-d[t]) - V[t](1-d[t-1])   (done mask
//          of ppo.py:387 applied on the fly; optionally written out)
//   pass 2 (item = (segment, window), LG lanes per item, window index fixed
//          per thread): ret = sum g[k] r[s+k] + Vm[s+H] gamma^H,
//          adv = sum (td[s+k] g[k]) l[k]; LG > 1 splits long (non-RNN) windows.
struct GaeWinArgs {
  const float* values; float* values_masked; const float *rewards, *dones;
  int64_t B; int T, H, E, SB, LG, TPR;
  const float *gtab, *ltab; float gamma, gamma_H;
  float *adv, *ret; double* partials;
};

__device__ __forceinline__ void stage_f32(const float* __restrict__ src, float* __restrict__ dst,
                                          int n, bool vec) {
  if (vec) {
    const int n4 = n >> 2;
    const float4* s4 = reinterpret_cast<const float4*>(src);
    float4* d4 = reinterpret_cast<float4*>(dst);
    int i = threadIdx.x;
    for (; i + 3 * kWG < n4; i += 4 * kWG) {
      const float4 a = s4[i], b = s4[i + kWG], c = s4[i + 2 * kWG], d = s4[i + 3 * kWG];
      d4[i] = a; d4[i + kWG] = b; d4[i + 2 * kWG] = c; d4[i + 3 * kWG] = d;
    }
    for (; i < n4; i += kWG) d4[i] = s4[i];
    for (int j = (n4 << 2) + threadIdx.x; j < n; j += kWG) dst[j] = src[j];
  } else {
    for (int j = threadIdx.x; j < n; j += kWG) dst[j] = src[j];
  }
}

// Register prefetch of one full segment block ([r | d | V] as float4s, at most
// GAE_PF per thread): the next block's loads are in flight while the current
// block computes, so HBM sees a continuous stream.
constexpr int GAE_PF = 8;   // the SMI_GAE_PF_* macros below are unrolled for 8

// (8 named registers rather than an array: the compiler kept an array in scratch)
#define SMI_GAE_PF_LOAD(j)                                               \
  {                                                                      \
    const int q = threadIdx.x + (j) * kWG;                               \
    const float4* src = q < pf_nr4 ? pf_r4 : (q < 2 * pf_nr4 ? pf_d4 : pf_v4); \
    if (q < pf_tot4) pf##j = src[q];                                     \
  }
#define SMI_GAE_PREFETCH(b0)                                                                   \
  {                                                                                            \
    const float4* pf_r4 = reinterpret_cast<const float4*>(a.rewards + (b0) * T);               \
    const float4* pf_d4 = reinterpret_cast<const float4*>(a.dones + (b0) * T) - pf_nr4;        \
    const float4* pf_v4 = reinterpret_cast<const float4*>(a.values + (b0) * T1) - 2 * pf_nr4;  \
    SMI_GAE_PF_LOAD(0) SMI_GAE_PF_LOAD(1) SMI_GAE_PF_LOAD(2) SMI_GAE_PF_LOAD(3)                \
    SMI_GAE_PF_LOAD(4) SMI_GAE_PF_LOAD(5) SMI_GAE_PF_LOAD(6) SMI_GAE_PF_LOAD(7)                \
  }
#define SMI_GAE_PF_STORE(j)                                              \
  {                                                                      \
    const int q = threadIdx.x + (j) * kWG;                               \
    if (q < pf_tot4) l4[q] = pf##j;                                      \
  }

__global__ void __launch_bounds__(kWG)
gae_windows_kernel(GaeWinArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  __shared__ double red[kNW];
  const int T = a.T, T1 = T + 1, H = a.H, E = a.E, LG = a.LG, TPR = a.TPR;
  const int SBT4 = (a.SB * T + 3) & ~3, SBT14 = (a.SB * T1 + 3) & ~3;
  float* sr = sm;                         // [SB*T] rewards
  float* sd = sr + SBT4;                  // [SB*T] dones
  float* sv = sd + SBT4;                  // [SB*T1] values (raw)
  float* st = sv + SBT14;                 // [SB*T] td
  float* sg = st + SBT4;                  // [H] gamma table
  float* sl = sg + H;                     // [H] lambda table
  for (int k = threadIdx.x; k < H; k += kWG) { sg[k] = a.gtab[k]; sl[k] = a.ltab[k]; }
  // pass-1 mapping: thread -> (row lane, t)
  const int tcol = threadIdx.x & (TPR - 1);
  const int trow = threadIdx.x / TPR;
  const int RPP = kWG / TPR;
  // pass-2 mapping: thread -> (segment offset, window w) fixed across passes
  const int lane_g = threadIdx.x & (LG - 1);
  const int it0 = threadIdx.x / LG;
  const int SPP = (kWG / LG) / E;          // segments per pass (>= 1 by construction)
  const int s_off = it0 / E, w = it0 - s_off * E;
  const bool p2_active = s_off < SPP;
  double psum = 0.0, psq = 0.0;
  const int64_t nblk = (a.B + a.SB - 1) / a.SB;
  const bool vec = ((reinterpret_cast<uintptr_t>(a.rewards) | reinterpret_cast<uintptr_t>(a.dones) |
                     reinterpret_cast<uintptr_t>(a.values)) & 15) == 0;
  const float gamma = a.gamma;
  // full blocks (nseg == SB, 16-byte aligned arrays) go through the register
  // prefetch; the ragged last block is staged directly
  const int64_t nfull = vec ? a.B / a.SB : 0;
  const int nr4 = a.SB * T / 4, nv4 = a.SB * T1 / 4;
  const int pf_nr4 = nr4, pf_tot4 = 2 * nr4 + nv4;
  float4 pf0, pf1, pf2, pf3, pf4, pf5, pf6, pf7;
  if (blockIdx.x < nfull) SMI_GAE_PREFETCH((int64_t)blockIdx.x * a.SB)
  for (int64_t blk = blockIdx.x; blk < nblk; blk += gridDim.x) {
    const int64_t b0 = blk * a.SB;
    const int nseg = (int)min((int64_t)a.SB, a.B - b0);
    __syncthreads();
    if (blk < nfull) {
      // sr, sd, sv are contiguous in LDS (SB*T is a multiple of 4)
      float4* l4 = reinterpret_cast<float4*>(sr);
      SMI_GAE_PF_STORE(0) SMI_GAE_PF_STORE(1) SMI_GAE_PF_STORE(2) SMI_GAE_PF_STORE(3)
      SMI_GAE_PF_STORE(4) SMI_GAE_PF_STORE(5) SMI_GAE_PF_STORE(6) SMI_GAE_PF_STORE(7)
      const int64_t nxt = blk + gridDim.x;
      if (nxt < nfull) SMI_GAE_PREFETCH(nxt * a.SB)
    } else {
      stage_f32(a.rewards + b0 * T, sr, nseg * T, vec);
      stage_f32(a.dones + b0 * T, sd, nseg * T, vec);
      stage_f32(a.values + b0 * T1, sv, nseg * T1, vec);
    }
    __syncthreads();
    for (int s = trow; s < nseg; s += RPP) {
      const float* r = sr + s * T;
      const float* d = sd + s * T;
      const float* v = sv + s * T1;
      for (int t = tcol; t < T1; t += TPR) {
        const float vm = t > 0 ? v[t] * (1.f - d[t - 1]) : v[0];
        if (a.values_masked) a.values_masked[(b0 + s) * T1 + t] = vm;
        if (t < T) {
          const float vm1 = v[t + 1] * (1.f - d[t]);
          st[s * T + t] = (r[t] + gamma * vm1) - vm;
        }
      }
    }
    __syncthreads();
    if (p2_active) {
      for (int s = s_off; s < nseg; s += SPP) {
        const float* r = sr + s * T + w;
        const float* td = st + s * T + w;
        float rs = 0.f, as = 0.f;
        for (int k = lane_g; k < H; k += LG) {
          rs += sg[k] * r[k];
          as += (td[k] * sg[k]) * sl[k];
        }
        for (int o = LG >> 1; o > 0; o >>= 1) {
          rs += __shfl_xor(rs, o, 64);
          as += __shfl_xor(as, o, 64);
        }
        if (lane_g == 0) {
          const float vH = sv[s * T1 + w + H] * (1.f - sd[s * T + w + H - 1]);
          const int64_t o = (b0 + s) * E + w;
          a.ret[o] = rs + vH * a.gamma_H;
          a.adv[o] = as;
          psum += (double)as;
          psq += (double)as * (double)as;
        }
      }
    }
  }
  const double s1 = block_sum_d(psum, red);
  const double s2 = block_sum_d(psq, red);
  if (threadIdx.x == 0 && a.partials) {
    a.partials[2 * blockIdx.x] = s1;
    a.partials[2 * blockIdx.x + 1] = s2;
  }
}

// ---------------------------------------------------- lane-per-step variant
// For T + 1 <= 64 (every BASELINE config): no LDS, no barriers.  A segment row
// is mapped onto TPR = 2^k >= T+1 lanes of a wave (lane t holds step t), so a
// wave's loads of r, d, V cover 64/TPR consecutive segments — contiguous
// memory, coalesced — and U row groups are loaded before any is used (24
// loads in flight per lane).  Neighbouring steps come from lane shuffles:
//   V[t+1] <- lane t+1,  d[t-1] <- lane t-1,
//   td_t = r_t + gamma * V[t+1](1-d[t]) - V[t](1-d[t-1])    (ppo.py:387,390)
// Windows: E == 1 (non-RNN, H == T) is a lane reduction over the row; E > 1
// (RNN, H <= 16) sums H shuffled-down terms, lane w writing window w.
template <int TPR>
__global__ void __launch_bounds__(kWG)
gae_rows_kernel(GaeWinArgs a) {
  constexpr int RPW = 64 / TPR;           // segment rows per wave-row-group
  constexpr int U = 8;                    // row groups in flight per wave
  __shared__ double red[kNW];
  const int T = a.T, T1 = T + 1, H = a.H, E = a.E;
  const int lane = threadIdx.x & 63;
  const int t = lane & (TPR - 1);
  const int rsub = lane / TPR;
  const int64_t nwaves = (int64_t)gridDim.x * kNW;
  const int64_t wid = (int64_t)blockIdx.x * kNW + (threadIdx.x >> 6);
  const int64_t ngroups = (a.B + RPW - 1) / RPW;
  const float gamma = a.gamma, gamma_H = a.gamma_H;
  // per-lane window coefficients: lane t needs g[t], l[t] (E == 1) or the
  // whole H-table (E > 1, read from the constant tables in the loop)
  const float gt_raw = a.gtab[t < H ? t : H - 1], lt_raw = a.ltab[t < H ? t : H - 1];
  const float gt = t < H ? gt_raw : 0.f;
  const float lt = t < H ? lt_raw : 0.f;
  double psum = 0.0, psq = 0.0;
  for (int64_t g0 = wid; g0 < ngroups; g0 += U * nwaves) {
    float r[U], d[U], v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      // unconditional loads from clamped addresses (a predicated load makes
      // hipcc branch and wait per element); out-of-range lanes are zeroed after
      const int64_t row = (g0 + u * nwaves) * RPW + rsub;
      const int64_t rr = row < a.B ? row : a.B - 1;
      const int tc = t < T ? t : T - 1, tv = t < T1 ? t : T;
      r[u] = a.rewards[rr * T + tc];
      d[u] = a.dones[rr * T + tc];
      v[u] = a.values[rr * T1 + tv];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (t >= T) { r[u] = 0.f; d[u] = 0.f; }
      if (t >= T1) v[u] = 0.f;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t row = (g0 + u * nwaves) * RPW + rsub;
      const float v1 = __shfl_down(v[u], 1, TPR);       // V[t+1]
      const float dm1 = __shfl_up(d[u], 1, TPR);        // d[t-1]
      const float vm = t > 0 ? v[u] * (1.f - dm1) : v[u];
      const float vm1 = v1 * (1.f - d[u]);
      if (a.values_masked && row < a.B && t < T1) a.values_masked[row * T1 + t] = vm;
      const float td = t < T ? (r[u] + gamma * vm1) - vm : 0.f;
      if (E == 1) {
        float rs = gt * r[u];
        float as = (td * gt) * lt;
#pragma unroll
        for (int o = TPR >> 1; o > 0; o >>= 1) {
          rs += __shfl_xor(rs, o, TPR);
          as += __shfl_xor(as, o, TPR);
        }
        const float vH = __shfl(vm, H, TPR);              // Vm[H]
        if (t == 0 && row < a.B) {
          a.ret[row] = rs + vH * gamma_H;
          a.adv[row] = as;
          psum += (double)as;
          psq += (double)as * (double)as;
        }
      } else {
        float rs = 0.f, as = 0.f;
        for (int k = 0; k < H; ++k) {
          const float rk = __shfl_down(r[u], k, TPR);
          const float tk = __shfl_down(td, k, TPR);
          const float gk = __shfl(gt, k, TPR), lk = __shfl(lt, k, TPR);
          rs += gk * rk;
          as += (tk * gk) * lk;
        }
        const float vH = __shfl_down(vm, H, TPR);         // Vm[w+H]
        if (t < E && row < a.B) {
          const int64_t o = row * E + t;
          a.ret[o] = rs + vH * gamma_H;
          a.adv[o] = as;
          psum += (double)as;
          psq += (double)as * (double)as;
        }
      }
    }
  }
  const double s1 = block_sum_d(psum, red);
  const double s2 = block_sum_d(psq, red);
  if (threadIdx.x == 0 && a.partials) {
    a.partials[2 * blockIdx.x] = s1;
    a.partials[2 * blockIdx.x + 1] = s2;
  }
}

// ------------------------------------------------ segment-per-thread variant
// The RNN windows of the reference defaults (n_step T, horizon H compile-time;
// ppo_configs.py: 25 / 5).  A workgroup owns SEG = 256 consecutive segments,
// one per thread.  Their r, d, V are contiguous in HBM ([SEG][T], [SEG][T],
// [SEG][T+1]) and move as ONE stream of 16-byte loads into LDS, register-
// prefetched one block ahead; each thread then runs its row from LDS (stride
// T floats: conflict-free for odd T) with the window sums in registers
// (fully unrolled, H-deep ring), and the block's adv/ret leave through LDS as
// 16-byte coalesced stores.  Same fp32 op order as gae_rows_kernel.
template <int T, int H, int SEG_>
struct GaeSeg {
  static constexpr int SEG = SEG_, T1 = T + 1, E = T - H + 1;
  static constexpr int NF4 = SEG * (3 * T + 1) / 4;            // float4s of one block
  static constexpr int NPF = (NF4 + SEG - 1) / SEG;            // per thread
  static constexpr size_t LDS = ((size_t)SEG * (3 * T + 1) + 2 * H) * 4;   // + gamma/lambda tables
};

template <int T, int H, int SEG_>
__global__ void __launch_bounds__(SEG_)
gae_seg_kernel(GaeWinArgs a, int64_t nblocks) {
  using G = GaeSeg<T, H, SEG_>;
  constexpr int SEG = G::SEG, T1 = G::T1, E = G::E, NPF = G::NPF, NF4 = G::NF4;
  constexpr int NT = SEG;                                       // threads = segments
  constexpr int NR4 = SEG * T / 4;                              // float4s of r (and of d)
  extern __shared__ __attribute__((aligned(16))) float sm[];
  __shared__ double red[NT / 64];
  float* sr = sm;                  // [SEG][T]
  float* sd = sr + SEG * T;        // [SEG][T]
  float* sv = sd + SEG * T;        // [SEG][T1]
  const int tid = threadIdx.x;
  float* sg = sv + SEG * T1;       // [H] gamma^k, [H] lambda^k (E == 1 reads them per step)
  for (int k = tid; k < H; k += NT) { sg[k] = a.gtab[k]; sg[H + k] = a.ltab[k]; }
  constexpr int HK = E > 1 ? H : 1;
  float gk[HK], lk[HK];
#pragma unroll
  for (int k = 0; k < HK; ++k) { gk[k] = a.gtab[k]; lk[k] = a.ltab[k]; }
  const float gamma = a.gamma, gamma_H = a.gamma_H;
  double psum = 0.0, psq = 0.0;
  // prefetch registers as named variables (an indexed float4 array stays in
  // scratch whatever its shape)
  static_assert(NPF <= 40, "gae_seg: prefetch depth");
#define SMI_GAE_X24(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) \
  X(13) X(14) X(15) X(16) X(17) X(18) X(19) X(20) X(21) X(22) X(23) X(24) X(25) X(26)   \
  X(27) X(28) X(29) X(30) X(31) X(32) X(33) X(34) X(35) X(36) X(37) X(38) X(39)
#define SMI_GAE_DECL(j) float4 pf##j = make_float4(0.f, 0.f, 0.f, 0.f);
  SMI_GAE_X24(SMI_GAE_DECL)
#define SMI_GAE_LD(j)                                                          \
  if ((j) < NPF) {                                                             \
    const int q = tid + (j) * NT;                                              \
    const float4* src = q < NR4 ? r4 : (q < 2 * NR4 ? d4 : v4);                \
    if (q < NF4) pf##j = src[q];                                               \
  }
#define SMI_GAE_ST(j)                                                          \
  if ((j) < NPF) {                                                             \
    const int q = tid + (j) * NT;                                              \
    if (q < NF4) l4[q] = pf##j;                                                \
  }
#define SMI_GAE_SEG_PREFETCH(BLK)                                                              \
  {                                                                                            \
    const float4* r4 = reinterpret_cast<const float4*>(a.rewards + (BLK) * SEG * T);           \
    const float4* d4 = reinterpret_cast<const float4*>(a.dones + (BLK) * SEG * T) - NR4;       \
    const float4* v4 = reinterpret_cast<const float4*>(a.values + (BLK) * SEG * T1) - 2 * NR4; \
    SMI_GAE_X24(SMI_GAE_LD)                                                                    \
  }
  if (blockIdx.x < nblocks) SMI_GAE_SEG_PREFETCH((int64_t)blockIdx.x)
  for (int64_t blk = blockIdx.x; blk < nblocks; blk += gridDim.x) {
    __syncthreads();                        // previous block's outputs have left LDS
    {
      float4* l4 = reinterpret_cast<float4*>(sm);
      SMI_GAE_X24(SMI_GAE_ST)
    }
    if (blk + gridDim.x < nblocks) SMI_GAE_SEG_PREFETCH(blk + gridDim.x)
    __syncthreads();
    // ---- one segment row per thread
    const float* r = sr + tid * T;
    const float* d = sd + tid * T;
    const float* v = sv + tid * T1;
    float adv[E], ret[E];
    constexpr int HR = E > 1 ? H : 1;
    float rr[HR], tt[HR];                  // ring: index k = step (t - H + 1 + k)
    float rs1 = 0.f, as1 = 0.f;            // E == 1: the single window, summed in k order
    float vm = v[0];                       // Vm[t]
    float dprev = 0.f;
    // E > 1: fully unrolled (register-indexed windows); E == 1: partial unroll
    // keeps the row's LDS reads from being hoisted into registers all at once
#pragma unroll (E > 1 ? T : 5)
    for (int t = 0; t < T; ++t) {
      const float rt = r[t], dt = d[t];
      if (t > 0) vm = v[t] * (1.f - dprev);
      const float vm1 = v[t + 1] * (1.f - dt);
      if (a.values_masked) a.values_masked[(blk * SEG + tid) * T1 + t] = vm;
      const float td = (rt + gamma * vm1) - vm;
      if constexpr (E == 1) {
        const float g = sg[t], l = sg[H + t];
        rs1 += g * rt;
        as1 += (td * g) * l;
        if (t == T - 1) {
          ret[0] = rs1 + vm1 * gamma_H;
          adv[0] = as1;
          psum += (double)as1;
          psq += (double)as1 * (double)as1;
        }
      } else {
#pragma unroll
      for (int k = 0; k < H - 1; ++k) { rr[k] = rr[k + 1]; tt[k] = tt[k + 1]; }
      rr[H - 1] = rt;
      tt[H - 1] = td;
      if (t >= H - 1) {
        float rs = 0.f, as = 0.f;
#pragma unroll
        for (int k = 0; k < H; ++k) {
          rs += gk[k] * rr[k];
          as += (tt[k] * gk[k]) * lk[k];
        }
        // window w = t - H + 1 needs Vm[w + H] = Vm[t + 1]
        ret[t - H + 1] = rs + vm1 * gamma_H;
        adv[t - H + 1] = as;
        psum += (double)as;
        psq += (double)as * (double)as;
      }
      }
      dprev = dt;
    }
    if (a.values_masked) a.values_masked[(blk * SEG + tid) * T1 + T] = v[T] * (1.f - dprev);
    __syncthreads();                        // every row has been read
    float* oa = sr;                         // [SEG][E] adv   (E <= T)
    float* orr = sd;                        // [SEG][E] ret
#pragma unroll
    for (int w = 0; w < E; ++w) { oa[tid * E + w] = adv[w]; orr[tid * E + w] = ret[w]; }
    __syncthreads();
    {
      constexpr int NO4 = SEG * E / 4;
      float4* ga = reinterpret_cast<float4*>(a.adv + blk * SEG * E);
      float4* gr = reinterpret_cast<float4*>(a.ret + blk * SEG * E);
      const float4* la = reinterpret_cast<const float4*>(oa);
      const float4* lr = reinterpret_cast<const float4*>(orr);
      for (int q = tid; q < NO4; q += NT) { ga[q] = la[q]; gr[q] = lr[q]; }
      if constexpr ((SEG * E) % 4 != 0) {
        for (int q = NO4 * 4 + tid; q < SEG * E; q += NT) {
          a.adv[blk * SEG * E + q] = oa[q];
          a.ret[blk * SEG * E + q] = orr[q];
        }
      }
    }
  }
#undef SMI_GAE_SEG_PREFETCH
#undef SMI_GAE_X24
#undef SMI_GAE_DECL
#undef SMI_GAE_LD
#undef SMI_GAE_ST
  const double s1 = block_sum_d<NT>(psum, red);
  const double s2 = block_sum_d<NT>(psq, red);
  if (threadIdx.x == 0 && a.partials) {
    a.partials[2 * blockIdx.x] = s1;
    a.partials[2 * blockIdx.x + 1] = s2;
  }
}

// Launch the segment-per-thread kernel over the full 256-segment blocks; the
// ragged tail goes to gae_rows_kernel (partials appended).  Returns false when
// (T, H) has no instantiation or the buffers are not 16-byte aligned.
template <int T, int H, int SEG>
static bool try_gae_seg(const GaeWinArgs& a, int* n_partials, hipStream_t stream, int* rc) {
  using G = GaeSeg<T, H, SEG>;
  if (a.T != T || a.H != H) return false;
  const uintptr_t al = reinterpret_cast<uintptr_t>(a.rewards) | reinterpret_cast<uintptr_t>(a.dones) |
                       reinterpret_cast<uintptr_t>(a.values) | reinterpret_cast<uintptr_t>(a.adv) |
                       reinterpret_cast<uintptr_t>(a.ret);
  if (al & 15) return false;
  const int64_t nblk = a.B / G::SEG;
  if (nblk < 1) return false;
  auto k = gae_seg_kernel<T, H, SEG>;
  allow_lds(k, G::LDS);
  static int cap = 0;
  if (!cap) {
    cap = resident_grid(k, SEG, G::LDS);
    if (cap > 1024) cap = 1024;
    // SMI_GAE_GRID: workgroups of the grid-stride loop (each block's loads
    // prefetched behind the previous block's rows; A/B knob)
    const char* e = getenv("SMI_GAE_GRID");
    const int g = e && e[0] ? atoi(e) : 0;
    if (g > 0 && g < cap) cap = g;
  }
  const int grid = (int)(nblk < cap ? nblk : cap);
  hipLaunchKernelGGL(k, dim3(grid), dim3(SEG), G::LDS, stream, a, nblk);
  *rc = check_launch("gae_seg_kernel");
  if (*rc) return true;
  int np = grid;
  const int64_t done = nblk * G::SEG;
  if (done < a.B) {
    GaeWinArgs t = a;
    t.B = a.B - done;
    t.values = a.values + done * (T + 1);
    t.values_masked = a.values_masked ? a.values_masked + done * (T + 1) : nullptr;
    t.rewards = a.rewards + done * T;
    t.dones = a.dones + done * T;
    t.adv = a.adv + done * G::E;
    t.ret = a.ret + done * G::E;
    t.partials = a.partials ? a.partials + 2 * grid : nullptr;
    int TPR = 8;
    while (TPR < T + 1) TPR *= 2;
    const int64_t groups = (t.B + 64 / TPR - 1) / (64 / TPR);
    int g2 = (int)((groups + kNW * 8 - 1) / (kNW * 8));
    g2 = g2 < 1 ? 1 : (g2 > 1024 ? 1024 : g2);
    if (TPR == 32) hipLaunchKernelGGL(gae_rows_kernel<32>, dim3(g2), dim3(kWG), 0, stream, t);
    else hipLaunchKernelGGL(gae_rows_kernel<64>, dim3(g2), dim3(kWG), 0, stream, t);
    *rc = check_launch("gae_rows_kernel");
    np += g2;
  }
  if (n_partials) *n_partials = np;
  return true;
}

// ============================================================ host launchers
int launch_critic_gae(const float* critic_params, int D, int H1, int H2, int use_zf,
                      const float* zf_sum, const float* zf_sumsq, const float* zf_count,
                      float zf_eps, const float* obs, const float* obs_next,
                      const float* rewards, const float* dones, int B, int T,
                      const float* gtab, const float* ltab, float gamma, float gamma_T,
                      float* values, float* adv, float* ret, hipStream_t stream) {
  CriticGaeArgs a;
  a.params = critic_params; a.D = D; a.H1 = H1; a.H2 = H2;
  a.use_zf = use_zf; a.zf_sum = zf_sum; a.zf_sumsq = zf_sumsq; a.zf_count = zf_count;
  a.zf_eps = zf_eps;
  a.obs = obs; a.obs_next = obs_next; a.rewards = rewards; a.dones = dones;
  a.B = B; a.T = T;
  a.gtab = gtab; a.ltab = ltab; a.gamma = gamma; a.gamma_T = gamma_T;
  a.values = values; a.adv = adv; a.ret = ret;
  const int T1 = T + 1;
  // segments per chunk: values of a chunk stay in LDS (<= 4096 floats); aim
  // for >= 256 workgroups when the batch is large.
  int CS = 4096 / T1;
  if (CS < 1) CS = 1;
  const int64_t rows_total = (int64_t)B * T1;
  const int want_cs = (int)((rows_total + 256 * kRT - 1) / (256 * kRT) / T1) + 1;
  if (want_cs < CS) CS = want_cs;
  if (CS > B) CS = B;
  a.CS = CS;
  const MlpLayout L = mlp_layout(D, H1, H2, 1, 0);
  const int ldX = pad_ld(D), ldH1 = pad_ld(H1), ldH2 = pad_ld(H2), ldO = pad_small(1);
  int64_t base = 2 * round4(D) + kRT * (ldX + ldH1 + ldH2 + ldO) + round4(CS * T1);
  int64_t with_p = base + L.pcount;
  a.params_in_lds = (with_p * 4 <= 160 * 1024) ? 1 : 0;
  const int64_t lds = (a.params_in_lds ? with_p : base) * 4;
  if (lds > 160 * 1024) return set_error(SMI_E_NOFIT, "critic_gae: LDS does not fit");
  const int nchunks = (B + CS - 1) / CS;
  const int grid = nchunks < 2048 ? nchunks : 2048;
  allow_lds(critic_gae_kernel, (size_t)lds);
  hipLaunchKernelGGL(critic_gae_kernel, dim3(grid), dim3(kWG), (size_t)lds, stream, a);
  return check_launch("critic_gae_kernel");
}

int gae_windows_max_partials(int64_t B, int T) {
  (void)T;
  (void)B;
  return 2048;
}

int launch_gae_windows(const float* values, float* values_masked, const float* rewards,
                       const float* dones, int64_t B, int T, int H, const float* gtab,
                       const float* ltab, float gamma, float gamma_H, float* adv, float* ret,
                       double* partials, int* n_partials, hipStream_t stream) {
  if (H < 1 || H > T) return set_error(SMI_E_ARG, "gae_windows: horizon must be in [1, T]");
  GaeWinArgs a;
  a.values = values; a.values_masked = values_masked; a.rewards = rewards; a.dones = dones;
  a.B = B; a.T = T; a.H = H;
  a.E = T - H + 1;
  a.gtab = gtab; a.ltab = ltab; a.gamma = gamma; a.gamma_H = gamma_H;
  a.adv = adv; a.ret = ret; a.partials = partials;
  const bool faulted = fault() == SMI_FAULT_GAE_HORIZON && H > 1 && a.E > 1;
  if (faulted) {             // windows of H - 1 steps, the same E windows
    a.H = H - 1;
    a.gamma_H = gamma_H / gamma;
  }
  if (!faulted) {
    int rc = 0;
    // the reference defaults: RNN n_step 25 / horizon 5; non-RNN n_step 50
    // 64-segment workgroups (19.5 KB of LDS, one wave: several resident per
    // CU, so one block's stores overlap another's loads; 16 blocks at C3
    // instead of 4); SMI_GAE_SEG=256: the round-5 256-segment blocks (A/B)
    static const int seg = [] { const char* e = getenv("SMI_GAE_SEG"); return e && atoi(e) == 256 ? 256 : 64; }();
    if (seg == 64 && try_gae_seg<25, 5, 64>(a, n_partials, stream, &rc)) return rc;
    if (try_gae_seg<25, 5, 256>(a, n_partials, stream, &rc)) return rc;
    if (try_gae_seg<50, 50, 128>(a, n_partials, stream, &rc)) return rc;
  }
  if (T + 1 <= 64 && (a.E == 1 || H <= 16) && (!faulted || a.H <= 16)) {
    int TPR = 8;
    while (TPR < T + 1) TPR *= 2;
    const int64_t groups = (B + 64 / TPR - 1) / (64 / TPR);
    int64_t g = (groups + kNW * 8 - 1) / (kNW * 8);
    static int cap[4] = {0, 0, 0, 0};
    const int ci = TPR == 8 ? 0 : TPR == 16 ? 1 : TPR == 32 ? 2 : 3;
    if (!cap[ci]) {
      cap[ci] = TPR == 8 ? resident_grid(gae_rows_kernel<8>, kWG, 0)
              : TPR == 16 ? resident_grid(gae_rows_kernel<16>, kWG, 0)
              : TPR == 32 ? resident_grid(gae_rows_kernel<32>, kWG, 0)
                          : resident_grid(gae_rows_kernel<64>, kWG, 0);
      if (cap[ci] > 2048) cap[ci] = 2048;         // <= smi_gae_windows_max_partials
    }
    const int grid = (int)(g < cap[ci] ? (g < 1 ? 1 : g) : cap[ci]);
    if (TPR == 8) hipLaunchKernelGGL(gae_rows_kernel<8>, dim3(grid), dim3(kWG), 0, stream, a);
    else if (TPR == 16) hipLaunchKernelGGL(gae_rows_kernel<16>, dim3(grid), dim3(kWG), 0, stream, a);
    else if (TPR == 32) hipLaunchKernelGGL(gae_rows_kernel<32>, dim3(grid), dim3(kWG), 0, stream, a);
    else hipLaunchKernelGGL(gae_rows_kernel<64>, dim3(grid), dim3(kWG), 0, stream, a);
    if (n_partials) *n_partials = grid;
    return check_launch("gae_rows_kernel");
  }
  // lanes per window: split long windows so a block pass keeps every lane busy
  int LG = 1;
  while (LG < 16 && 2 * LG <= H / 3) LG *= 2;
  while (LG > 1 && (kWG / LG) < a.E) LG >>= 1;
  if ((kWG / LG) < a.E) return set_error(SMI_E_ARG, "gae_windows: more than 256 windows per segment");
  a.LG = LG;
  int TPR = 1;
  while (TPR < 64 && TPR < T + 1) TPR *= 2;
  a.TPR = TPR;
  // segments per block: ~1024 lane-items per pass, a multiple of 4 (16-byte
  // aligned staging), LDS <= 40 KB so several blocks share a CU
  int SB = (1024 + a.E * LG - 1) / (a.E * LG);
  int max_sb = (40 * 1024 / 4 - 2 * H - 16) / (4 * T + 1);
  const int max_pf = GAE_PF * kWG * 4 / (3 * T + 1);     // register prefetch capacity
  if (max_sb > max_pf) max_sb = max_pf;
  if (SB > max_sb) SB = max_sb;
  SB = SB & ~3;
  if (SB < 4) SB = 4;
  a.SB = SB;
  a.gtab = gtab; a.ltab = ltab; a.gamma = gamma; a.gamma_H = gamma_H;
  a.adv = adv; a.ret = ret; a.partials = partials;
  const int64_t nblk = (B + SB - 1) / SB;
  const int grid = (int)(nblk < 2048 ? nblk : 2048);
  const size_t lds = (size_t)(3 * ((SB * T + 3) & ~3) + ((SB * (T + 1) + 3) & ~3) + 2 * H) * 4;
  if (lds > 160 * 1024) return set_error(SMI_E_NOFIT, "gae_windows: T too large");
  allow_lds(gae_windows_kernel, lds);
  hipLaunchKernelGGL(gae_windows_kernel, dim3(grid), dim3(kWG), lds, stream, a);
  if (n_partials) *n_partials = grid;
  return check_launch("gae_windows_kernel");
}

}  // namespace smi
