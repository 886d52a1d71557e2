// psrt_device.h — device-side arithmetic of the hot path, in the reference's
// IEEE binary64 operation order. Compiled with -ffp-contract=off: every
// a*b+c below must stay a v_mul_f64 + v_add_f64 pair (an FMA changes the
// rounding, flips trapped/escaped paths and biases the image; SURVEY.md
// fact 5). Division and sqrt are the IEEE-correct gfx950 expansions.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace psrt {

// ---- counter RNG (reference draw site random.h:4-14) --------
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ULL;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

// The counter stream's generator: a sample's 64-bit
// state is {w: high word, x: low word}; each draw steps x by Marsaglia's
// xorshift32 (13, 17, 5), adds 0x9E3779B9 to w (a Weyl sequence, period 2^32
// per sample: distinct samples' xorshift runs that overlap still differ by
// their w), and returns raw = x + w; rand() = raw >> 1 (31 bits, the range of
// glibc rand()). 32-bit operations only: r05's PCG32 needed a 64-bit multiply
// per draw, and the look-ahead trials cost 3.5% more kernel time with it
// (profiles/r06_rngcost). A zero x stays zero (the draws are then the Weyl
// sequence alone), identically in the oracle and the reference's interposer.
constexpr uint32_t kWeyl = 0x9E3779B9u;

__device__ __forceinline__ uint32_t xorshift32(uint32_t x) {
  x ^= x << 13;
  x ^= x >> 17;
  x ^= x << 5;
  return x;
}

// One draw; returns rand().
__device__ __forceinline__ uint32_t rand31(uint64_t& st) {
  const uint32_t x = xorshift32((uint32_t)st);
  const uint32_t w = (uint32_t)(st >> 32) + kWeyl;
  st = ((uint64_t)w << 32) | x;
  return (x + w) >> 1;
}

// random_double(): (double)rand() / (RAND_MAX + 1.0). The divisor is 2^31, so
// the quotient is exact and equals the product with 2^-31.
__device__ __forceinline__ double random_double(uint64_t& st) {
  return (double)rand31(st) * 0x1p-31;
}

// Three consecutive raw draws (rand() = raw >> 1, see pm1_raw): the Weyl
// words of the three steps are independent adds; `next` is the state after
// the third draw.
__device__ __forceinline__ void raw32_x3(uint64_t s0, uint32_t& r0, uint32_t& r1, uint32_t& r2,
                                         uint64_t& next) {
  const uint32_t w = (uint32_t)(s0 >> 32);
  const uint32_t x1 = xorshift32((uint32_t)s0);
  const uint32_t x2 = xorshift32(x1);
  const uint32_t x3 = xorshift32(x2);
  r0 = x1 + (w + kWeyl);
  r1 = x2 + (w + 2u * kWeyl);
  r2 = x3 + (w + 3u * kWeyl);
  next = ((uint64_t)(w + 3u * kWeyl) << 32) | x3;
}

// random_double(-1, 1) = -1 + 2 * (rand() * 2^-31) (random.h:10-14) of the draw
// rand() = raw >> 1 is exactly (2 (raw >> 1) - 2^31) * 2^-31 (at most 32
// significant bits: neither the product nor the sum rounds). As an integer:
// 2 (raw >> 1) = raw & ~1, and subtracting 2^31 mod 2^32 flips the top bit
// (one v_bitop3_b32).
__device__ __forceinline__ int pm1_int_raw(uint32_t raw) {
  return (int)((raw & 0xFFFFFFFEu) ^ 0x80000000u);
}
// (double)pm1_int_raw(raw): with m = raw & ~1, the bits {hi 0x43300000, lo m}
// are the double 2^52 + m (exact), and (2^52 + m) - (2^52 + 2^31) = m - 2^31
// is exact (integers below 2^53, the difference below 2^31 in magnitude) and
// +0 when m = 2^31, as the conversion gives.
// (One FP64 add instead of a v_cvt_f64_i32.)
__device__ __forceinline__ double w_raw(uint32_t raw) {
  return __hiloint2double(0x43300000, (int)(raw & 0xFFFFFFFEu)) - 0x1.000008p52;
}
// pm1 = (m - 2^31) 2^-31 in one FP64 add: the bits {hi 0x41400000, lo m} are
// the double 2^21 + m 2^-31 (exact: m < 2^32 needs 31 fraction bits below
// 2^0, the format has 52 below 2^21), and (2^21 + m 2^-31) - (2^21 + 1) =
// m 2^-31 - 1 is exact (Sterbenz: the operands are within a factor of 2), +0
// when m = 2^31, as (double)pm1_int_raw(raw) * 2^-31 gives.
__device__ __forceinline__ double pm1_raw(uint32_t raw) {
  return __hiloint2double(0x41400000, (int)(raw & 0xFFFFFFFEu)) - 0x1.000008p21;
}

// random_in_unit_sphere's test !((x*x + y*y) + z*z > 1) (vec3.h:88) on
// x = w_x 2^-31 etc. (w: pm1_int_raw): every product and sum of the
// reference's expression is the same computation on w scaled by 2^-62 (power
// of two, no under/overflow: |w| <= 2^31), so rounding commutes with the
// scale and the test is !((wx*wx + wy*wy) + wz*wz > 2^62) on the doubles w.
__device__ __forceinline__ bool in_unit_sphere_raw(uint32_t x, uint32_t y, uint32_t z) {
  const double wx = w_raw(x), wy = w_raw(y), wz = w_raw(z);
  return !((wx * wx + wy * wy) + wz * wz > 0x1p62);
}

// The same test, decided in FP32 except within 2^-20 (relative) of the
// boundary: f = (float)w (RN, relative error <= 2^-24), S32 = fma(fx, fx,
// fma(fy, fy, fz*fz)) is within 2^-21 of S = wx^2 + wy^2 + wz^2 (all terms
// >= 0), and the reference's FP64 sum within 2^-51 of S. So S32 < 2^62
// (1 - 2^-20) puts the FP64 sum below 2^62 (inside) and S32 > 2^62
// (1 + 2^-20) above it (outside); the rest (~1.5e-6 of the trials) take the
// FP64 test, behind a wave-uniform branch.
__device__ __forceinline__ bool in_unit_sphere_raw_f32(uint32_t x, uint32_t y, uint32_t z) {
  const float fx = (float)pm1_int_raw(x), fy = (float)pm1_int_raw(y), fz = (float)pm1_int_raw(z);
  const float s = __builtin_fmaf(fx, fx, __builtin_fmaf(fy, fy, fz * fz));
  bool in = s < 0x1p62f * (1.0f - 0x1p-20f);
  const bool undecided = !in && !(s > 0x1p62f * (1.0f + 0x1p-20f));
  if (__builtin_expect(__ballot(undecided) != 0, 0)) {
    if (undecided) in = in_unit_sphere_raw(x, y, z);
  }
  return in;
}

}  // namespace psrt
