// sampler_kernels.hip — CPython-exact uniform replay index sampling and the
// replay row gather (UniformReplay.sample, surreal/replay/uniform_replay.py:43-47).
//
// The reference draws [random.randint(0, n-1) for _ in range(B)] from the
// Python stdlib generator: MT19937 (Matsumoto & Nishimura 1998) seeded by
// init_by_array with the 32-bit little-endian limbs of |seed|, and
// randint -> randrange -> _randbelow(n): k = n.bit_length(),
// r = genrand_uint32() >> (32 - k), rejected while r >= n (k <= 32 here, so one
// 32-bit word per attempt).  State: 624 words + position (625 uint32).
//
// Device algorithm (one workgroup of 1024 threads): the 624-word twist is done
// in its three dependency phases ([0,227) from old words, [227,454) and
// [454,623) from freshly twisted words 227 back, then word 623); tempering and
// the accept test are per-word parallel; a block prefix sum over accept flags
// places the accepted draws in stream order, so the output is the same
// sequence CPython produces, and exactly as many words are consumed.
#include "smi_device.hpp"
#include "smi_internal.hpp"

namespace smi {

constexpr int kMtN = 624, kMtM = 397;
constexpr uint32_t kMatA = 0x9908b0dfU, kUpper = 0x80000000U, kLower = 0x7fffffffU;

__host__ __device__ inline uint32_t mt_temper(uint32_t y) {
  y ^= (y >> 11);
  y ^= (y << 7) & 0x9d2c5680U;
  y ^= (y << 15) & 0xefc60000U;
  y ^= (y >> 18);
  return y;
}
__host__ __device__ inline uint32_t mt_mix(uint32_t hi, uint32_t lo, uint32_t far) {
  const uint32_t y = (hi & kUpper) | (lo & kLower);
  return far ^ (y >> 1) ^ ((y & 1U) ? kMatA : 0U);
}

// ------------------------------------------------------------------ host
static void mt_init_genrand(uint32_t* mt, uint32_t s) {
  mt[0] = s;
  for (int i = 1; i < kMtN; ++i) mt[i] = 1812433253U * (mt[i - 1] ^ (mt[i - 1] >> 30)) + (uint32_t)i;
}

void mt_seed_host(uint64_t seed, uint32_t* st) {
  uint32_t key[2];
  int klen;
  key[0] = (uint32_t)(seed & 0xffffffffULL);
  key[1] = (uint32_t)(seed >> 32);
  klen = key[1] ? 2 : 1;
  uint32_t* mt = st;
  mt_init_genrand(mt, 19650218U);
  int i = 1, j = 0;
  for (int k = (kMtN > klen ? kMtN : klen); k; --k) {
    mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1664525U)) + key[j] + (uint32_t)j;
    ++i; ++j;
    if (i >= kMtN) { mt[0] = mt[kMtN - 1]; i = 1; }
    if (j >= klen) j = 0;
  }
  for (int k = kMtN - 1; k; --k) {
    mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1566083941U)) - (uint32_t)i;
    ++i;
    if (i >= kMtN) { mt[0] = mt[kMtN - 1]; i = 1; }
  }
  mt[0] = 0x80000000U;
  st[kMtN] = kMtN;  // position: next call twists
}

static uint32_t mt_next_host(uint32_t* st) {
  uint32_t* mt = st;
  if (st[kMtN] >= (uint32_t)kMtN) {
    int kk = 0;
    for (; kk < kMtN - kMtM; ++kk) mt[kk] = mt_mix(mt[kk], mt[kk + 1], mt[kk + kMtM]);
    for (; kk < kMtN - 1; ++kk) mt[kk] = mt_mix(mt[kk], mt[kk + 1], mt[kk + (kMtM - kMtN)]);
    mt[kMtN - 1] = mt_mix(mt[kMtN - 1], mt[0], mt[kMtM - 1]);
    st[kMtN] = 0;
  }
  return mt_temper(mt[st[kMtN]++]);
}

static int bit_length(uint64_t n) {
  int k = 0;
  while (n) { ++k; n >>= 1; }
  return k;
}

int mt_randint_host(uint32_t* st, int64_t n, int64_t batch, int64_t* out) {
  const int k = bit_length((uint64_t)n);
  for (int64_t b = 0; b < batch; ++b) {
    uint32_t r;
    do { r = mt_next_host(st) >> (32 - k); } while ((int64_t)r >= n);
    out[b] = (int64_t)r;
  }
  return SMI_OK;
}

// ---------------------------------------------------------------- device
constexpr int kMtWG = 1024;

__global__ void __launch_bounds__(kMtWG)
mt_randint_kernel(uint32_t* __restrict__ st, int64_t n, int k, int64_t batch,
                  int64_t* __restrict__ out) {
  __shared__ uint32_t mt[kMtN];
  __shared__ int wsum[kMtWG / 64];
  __shared__ int s_pos;
  const int tid = threadIdx.x;
  for (int i = tid; i < kMtN; i += kMtWG) mt[i] = st[i];
  if (tid == 0) s_pos = (int)st[kMtN];
  __syncthreads();
  int64_t filled = 0;
  while (filled < batch) {
    if (s_pos >= kMtN) {
      // phase 1: [0, 227) from old words
      uint32_t nv = 0;
      if (tid < kMtN - kMtM) nv = mt_mix(mt[tid], mt[tid + 1], mt[tid + kMtM]);
      __syncthreads();
      if (tid < kMtN - kMtM) mt[tid] = nv;
      __syncthreads();
      // phase 2: [227, 454) and phase 3: [454, 623) read words 227 back
      for (int base = kMtN - kMtM; base < kMtN - 1; base += kMtN - kMtM) {
        const int kk = base + tid;
        const int end = (base + (kMtN - kMtM) < kMtN - 1) ? base + (kMtN - kMtM) : kMtN - 1;
        nv = 0;
        if (kk < end) nv = mt_mix(mt[kk], mt[kk + 1], mt[kk + (kMtM - kMtN)]);
        __syncthreads();
        if (kk < end) mt[kk] = nv;
        __syncthreads();
      }
      if (tid == 0) {
        mt[kMtN - 1] = mt_mix(mt[kMtN - 1], mt[0], mt[kMtM - 1]);
        s_pos = 0;
      }
      __syncthreads();
    }
    const int pos = s_pos;
    const int avail = kMtN - pos;
    // accept test per word in stream order
    int acc = 0;
    int64_t r = 0;
    if (tid < avail) {
      r = (int64_t)(mt_temper(mt[pos + tid]) >> (32 - k));
      acc = r < n ? 1 : 0;
    }
    // block exclusive scan of acc
    const int lane = tid & 63, wave = tid >> 6;
    const unsigned long long bal = __ballot(acc);
    const int wpre = __popcll(bal & ((1ULL << lane) - 1ULL));
    if (lane == 0) wsum[wave] = __popcll(bal);
    __syncthreads();
    int before = 0, total = 0;
    for (int w = 0; w < kMtWG / 64; ++w) {
      if (w < wave) before += wsum[w];
      total += wsum[w];
    }
    const int rank = before + wpre;
    const int64_t need = batch - filled;
    if (acc && rank < need) out[filled + rank] = r;
    // words consumed: all available, or up to the word giving the need-th draw
    __syncthreads();
    if (total >= need) {
      if (acc && rank == need - 1) s_pos = pos + tid + 1;
      __syncthreads();
      filled = batch;
    } else {
      if (tid == 0) s_pos = kMtN;
      __syncthreads();
      filled += total;
    }
    __syncthreads();
  }
  for (int i = tid; i < kMtN; i += kMtWG) st[i] = mt[i];
  if (tid == 0) st[kMtN] = (uint32_t)s_pos;
}

int launch_mt_randint(uint32_t* st, int64_t n, int64_t batch, int64_t* out, hipStream_t s) {
  if (n < 1 || n > 0xffffffffLL) return set_error(SMI_E_ARG, "mt_randint: n must be in [1, 2^32]");
  if (batch <= 0) return SMI_OK;
  const int k = bit_length((uint64_t)n);
  hipLaunchKernelGGL(mt_randint_kernel, dim3(1), dim3(kMtWG), 0, s, st, n, k, batch, out);
  return check_launch("mt_randint_kernel");
}

// ------------------------------------------------------------ row gather
// out[i][:] = table[idx[i]][:].  Output-ordered (coalesced stores); 16-byte
// elements when rows are float4-aligned, 32-bit index arithmetic when the
// output fits (a 64-bit divide per element costs more than the load), and four
// independent loads in flight per thread.
template <typename V, typename I>
__device__ __forceinline__ void gather_body(const V* __restrict__ table, I cols,
                                            const int64_t* __restrict__ idx, I total,
                                            V* __restrict__ out) {
  const I stride = (I)gridDim.x * kWG;
  I e = (I)blockIdx.x * kWG + threadIdx.x;
  for (; e + 3 * stride < total; e += 4 * stride) {
    V v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const I f = e + u * stride;
      const I i = f / cols, c = f - i * cols;
      v[u] = table[idx[i] * (int64_t)cols + c];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) out[e + u * stride] = v[u];
  }
  for (; e < total; e += stride) {
    const I i = e / cols, c = e - i * cols;
    out[e] = table[idx[i] * (int64_t)cols + c];
  }
}

__global__ void __launch_bounds__(kWG)
gather_rows_kernel(const float* __restrict__ table, int64_t cols, const int64_t* __restrict__ idx,
                   int64_t batch, float* __restrict__ out) {
  const uintptr_t al = reinterpret_cast<uintptr_t>(table) | reinterpret_cast<uintptr_t>(out);
  const bool v4 = (cols & 3) == 0 && (al & 15) == 0;
  // even widths (the DDPG row [s | a | r | s' | d] of HalfCheetah is 42 floats)
  // move as 8-byte elements
  const bool v2 = !v4 && (cols & 1) == 0 && (al & 7) == 0;
  const int64_t c = v4 ? cols >> 2 : v2 ? cols >> 1 : cols;
  const int64_t total = batch * c;
  if (total < ((int64_t)1 << 31)) {
    if (v4) gather_body<float4, uint32_t>(reinterpret_cast<const float4*>(table), (uint32_t)c, idx,
                                          (uint32_t)total, reinterpret_cast<float4*>(out));
    else if (v2) gather_body<float2, uint32_t>(reinterpret_cast<const float2*>(table), (uint32_t)c,
                                               idx, (uint32_t)total, reinterpret_cast<float2*>(out));
    else gather_body<float, uint32_t>(table, (uint32_t)c, idx, (uint32_t)total, out);
  } else {
    if (v4) gather_body<float4, int64_t>(reinterpret_cast<const float4*>(table), c, idx, total,
                                         reinterpret_cast<float4*>(out));
    else if (v2) gather_body<float2, int64_t>(reinterpret_cast<const float2*>(table), c, idx, total,
                                              reinterpret_cast<float2*>(out));
    else gather_body<float, int64_t>(table, c, idx, total, out);
  }
}

int launch_gather_rows(const float* table, int64_t cols, const int64_t* idx, int64_t batch,
                       float* out, hipStream_t s) {
  const int64_t work = batch * ((cols & 3) == 0 ? cols / 4 : (cols & 1) == 0 ? cols / 2 : cols);
  if (work <= 0) return SMI_OK;
  int64_t g = (work + kWG - 1) / kWG;
  g = (g + 3) / 4;
  if (g > 4096) g = 4096;
  if (g < 1) g = 1;
  hipLaunchKernelGGL(gather_rows_kernel, dim3((int)g), dim3(kWG), 0, s, table, cols, idx, batch, out);
  return check_launch("gather_rows_kernel");
}

}  // namespace smi
