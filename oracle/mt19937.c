/*
 * ORACLE (test infrastructure only — see oracle/__init__.py).
 *
 * Plain-C restatement of the index draw of UniformReplay.sample
 * (surreal/replay/uniform_replay.py:43-47):
 *     [random.randint(0, n - 1) for _ in range(batch)]
 * i.e. CPython's Mersenne Twister (Modules/_randommodule.c algorithm:
 * MT19937 of Matsumoto & Nishimura, init_by_array seeding from the 32-bit
 * little-endian limbs of |seed|) and Lib/random.py's
 * randint -> randrange -> _randbelow_with_getrandbits (k = n.bit_length(),
 * r = getrandbits(k) = genrand_uint32() >> (32 - k), rejected while r >= n).
 * Pinned against CPython `random` streams in tests/golden/sampler_streams.json.
 *
 * Build: make -C oracle   (-> oracle/_build/libmt_oracle.so)
 */
#include <stdint.h>

#define N 624
#define M 397

typedef struct {
  uint32_t mt[N];
  int index;
} mt_state;

static void init_genrand(mt_state* s, uint32_t seed) {
  s->mt[0] = seed;
  for (int i = 1; i < N; i++)
    s->mt[i] = 1812433253U * (s->mt[i - 1] ^ (s->mt[i - 1] >> 30)) + (uint32_t)i;
  s->index = N;
}

static void init_by_array(mt_state* s, const uint32_t* key, int klen) {
  init_genrand(s, 19650218U);
  int i = 1, j = 0;
  for (int k = (N > klen ? N : klen); k; k--) {
    s->mt[i] = (s->mt[i] ^ ((s->mt[i - 1] ^ (s->mt[i - 1] >> 30)) * 1664525U)) + key[j] + (uint32_t)j;
    i++;
    j++;
    if (i >= N) { s->mt[0] = s->mt[N - 1]; i = 1; }
    if (j >= klen) j = 0;
  }
  for (int k = N - 1; k; k--) {
    s->mt[i] = (s->mt[i] ^ ((s->mt[i - 1] ^ (s->mt[i - 1] >> 30)) * 1566083941U)) - (uint32_t)i;
    i++;
    if (i >= N) { s->mt[0] = s->mt[N - 1]; i = 1; }
  }
  s->mt[0] = 0x80000000U;
  s->index = N;
}

static uint32_t genrand_uint32(mt_state* s) {
  static const uint32_t mag01[2] = {0x0U, 0x9908b0dfU};
  uint32_t y;
  if (s->index >= N) {
    int kk;
    for (kk = 0; kk < N - M; kk++) {
      y = (s->mt[kk] & 0x80000000U) | (s->mt[kk + 1] & 0x7fffffffU);
      s->mt[kk] = s->mt[kk + M] ^ (y >> 1) ^ mag01[y & 1U];
    }
    for (; kk < N - 1; kk++) {
      y = (s->mt[kk] & 0x80000000U) | (s->mt[kk + 1] & 0x7fffffffU);
      s->mt[kk] = s->mt[kk + (M - N)] ^ (y >> 1) ^ mag01[y & 1U];
    }
    y = (s->mt[N - 1] & 0x80000000U) | (s->mt[0] & 0x7fffffffU);
    s->mt[N - 1] = s->mt[M - 1] ^ (y >> 1) ^ mag01[y & 1U];
    s->index = 0;
  }
  y = s->mt[s->index++];
  y ^= (y >> 11);
  y ^= (y << 7) & 0x9d2c5680U;
  y ^= (y << 15) & 0xefc60000U;
  y ^= (y >> 18);
  return y;
}

/* seed (|seed| < 2^64) then draw `batch` randint(0, n-1); n in [1, 2^32-1].
 * Returns the number of 32-bit words consumed. */
int64_t oracle_randint_stream(uint64_t seed, int64_t n, int64_t batch, int64_t* out) {
  mt_state s;
  uint32_t key[2] = {(uint32_t)(seed & 0xffffffffULL), (uint32_t)(seed >> 32)};
  init_by_array(&s, key, key[1] ? 2 : 1);
  int k = 0;
  for (uint64_t t = (uint64_t)n; t; t >>= 1) k++;
  int64_t words = 0;
  for (int64_t b = 0; b < batch; b++) {
    uint32_t r;
    do {
      r = genrand_uint32(&s) >> (32 - k);
      words++;
    } while ((int64_t)r >= n);
    out[b] = (int64_t)r;
  }
  return words;
}

/* state after seeding, in CPython getstate() order: 624 words + position */
void oracle_seed_state(uint64_t seed, uint32_t* out625) {
  mt_state s;
  uint32_t key[2] = {(uint32_t)(seed & 0xffffffffULL), (uint32_t)(seed >> 32)};
  init_by_array(&s, key, key[1] ? 2 : 1);
  for (int i = 0; i < N; i++) out625[i] = s.mt[i];
  out625[N] = (uint32_t)s.index;
}
