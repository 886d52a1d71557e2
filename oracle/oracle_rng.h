/*
 * ORACLE — test infrastructure only (never linked into libpsrt.so).
 *
 * The two random streams the oracle can drive the reference algorithm with.
 *
 * 1. GLIBC: a restatement of glibc 2.35's rand() (stdlib/random_r.c, TYPE_3
 *    additive-feedback generator, degree 31, separation 3) that the reference
 *    calls through random_double() (programs/random.h:4-8). The reference
 *    never calls srand(), so its state is glibc's default seed 1. Third-party
 *    dependency: glibc 2.35 (this image's libc); tests pin this restatement
 *    against the real rand().
 *
 * 2. COUNTER: the device contract. One stream per (pixel, sample):
 *                      key   = (uint64)(j*W + i) << 32 | s   (reference j:
 *                              0 = bottom row, main.cc:72; s = sample index)
 *                      state = splitmix64(key ^ splitmix64(seed))
 *    state = {w: high 32 bits, x: low 32 bits}; each draw steps
 *    x = xorshift32(x) (Marsaglia's 13, 17, 5), w += 0x9E3779B9, and rand()
 *    returns (x + w) >> 1 (31 bits, the range of glibc rand()), so the
 *    reference's random_double() = rand()/(RAND_MAX+1.0) maps it to [0,1)
 *    unchanged. (r01-r05: PCG32 XSH-RR; replaced in r06 by this 32-bit-op
 *    generator)
 *
 * random_double() here is the reference's INTENDED mapping
 * (double)rand() / (RAND_MAX + 1.0); the shipped random.h:7 computes
 * RAND_MAX + 1 in int, which overflows.
 */
#ifndef PSRT_ORACLE_RNG_H
#define PSRT_ORACLE_RNG_H

#include <stdint.h>

/* ---- glibc TYPE_3 (random_r.c: __srandom_r / __random_r) ---------------- */
typedef struct {
  int f, b; /* front / rear indices into the ring of 31 */
  int32_t ring[31];
} oracle_glibc_rand;

static inline void oracle_glibc_srand(oracle_glibc_rand* g, unsigned seed) {
  int32_t word;
  int i;
  if (seed == 0) seed = 1; /* random_r.c: "We must make sure the seed is not 0." */
  g->ring[0] = (int32_t)seed;
  word = (int32_t)seed;
  for (i = 1; i < 31; ++i) {
    /* word = 16807 * word % 2147483647, computed without overflow */
    long hi = word / 127773;
    long lo = word % 127773;
    word = (int32_t)(16807 * lo - 2836 * hi);
    if (word < 0) word += 2147483647;
    g->ring[i] = word;
  }
  g->f = 3; /* fptr = &state[SEP_3] */
  g->b = 0; /* rptr = &state[0]     */
  for (i = 0; i < 310; ++i) { /* kc * 10 discarded outputs */
    uint32_t v = (uint32_t)g->ring[g->f] + (uint32_t)g->ring[g->b];
    g->ring[g->f] = (int32_t)v;
    if (++g->f >= 31) g->f = 0;
    if (++g->b >= 31) g->b = 0;
  }
}

static inline int32_t oracle_glibc_next(oracle_glibc_rand* g) {
  uint32_t v = (uint32_t)g->ring[g->f] + (uint32_t)g->ring[g->b];
  g->ring[g->f] = (int32_t)v;
  if (++g->f >= 31) g->f = 0;
  if (++g->b >= 31) g->b = 0;
  return (int32_t)(v >> 1);
}

/* ---- counter stream ------------------------------------------------------- */
static inline uint64_t oracle_splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ULL;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

static inline uint64_t oracle_stream_state(uint64_t seed, uint32_t pixel,
                                           uint32_t sample) {
  uint64_t key = ((uint64_t)pixel << 32) | (uint64_t)sample;
  return oracle_splitmix64(key ^ oracle_splitmix64(seed));
}

/* one draw's raw 32 bits (rand() = raw >> 1); device: psrt_device.h rand31 */
static inline uint32_t oracle_counter_raw(uint64_t* state) {
  uint32_t x = (uint32_t)*state;
  uint32_t w = (uint32_t)(*state >> 32) + 0x9E3779B9u;
  x ^= x << 13;
  x ^= x >> 17;
  x ^= x << 5;
  *state = ((uint64_t)w << 32) | x;
  return x + w;
}

static inline int32_t oracle_counter_rand(uint64_t* state) {
  return (int32_t)(oracle_counter_raw(state) >> 1);
}

#endif /* PSRT_ORACLE_RNG_H */
