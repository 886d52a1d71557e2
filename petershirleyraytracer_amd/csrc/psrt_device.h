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

// PCG32 XSH-RR step; returns the 31-bit value the reference's rand() yields.
__device__ __forceinline__ uint32_t rand31(uint64_t& st) {
  const uint64_t old = st;
  st = old * 6364136223846793005ULL + 1442695040888963407ULL;
  const uint32_t xs = (uint32_t)(((old >> 18) ^ old) >> 27);
  const uint32_t rot = (uint32_t)(old >> 59);
  return ((xs >> rot) | (xs << ((32u - rot) & 31u))) >> 1;
}

// XSH-RR output of a PCG32 state (the value rand31 returns for `old`), >> 1.
__device__ __forceinline__ uint32_t pcg_out31(uint64_t old) {
  const uint32_t xs = (uint32_t)(((old >> 18) ^ old) >> 27);
  const uint32_t rot = (uint32_t)(old >> 59);
  return ((xs >> rot) | (xs << ((32u - rot) & 31u))) >> 1;
}

// Three consecutive draws with the LCG jumped ahead: s1 = a s0 + c,
// s2 = a^2 s0 + c (a + 1), s3 = a^3 s0 + c (a^2 + a + 1) (mod 2^64) — the same
// values as three rand31() calls, from independent multiplies. Returns the
// state after the third draw in `next`.
__device__ __forceinline__ void rand31_x3(uint64_t s0, uint32_t& r0, uint32_t& r1,
                                          uint32_t& r2, uint64_t& next) {
  const uint64_t s1 = s0 * 6364136223846793005ULL + 1442695040888963407ULL;
  const uint64_t s2 = s0 * 0x685f98a2018fade9ULL + 0x1a08ee1184ba6d32ULL;
  const uint64_t s3 = s0 * 0x0b046976f22528f5ULL + 0x9af678222e728119ULL;
  r0 = pcg_out31(s0);
  r1 = pcg_out31(s1);
  r2 = pcg_out31(s2);
  next = s3;
}

// random_double(): (double)rand() / (RAND_MAX + 1.0). The divisor is 2^31, so
// the quotient is exact and equals the product with 2^-31.
__device__ __forceinline__ double random_double(uint64_t& st) {
  return (double)rand31(st) * 0x1p-31;
}

// random_double(-1, 1) = -1 + (1 - -1) * random_double()   (random.h:10-14)
__device__ __forceinline__ double random_pm1(uint64_t& st) {
  return -1.0 + 2.0 * random_double(st);
}

// The same value from a raw rand() draw x: -1 + 2*(x*2^-31) is the exact
// value (2x - 2^31) * 2^-31 (at most 32 significant bits, so neither the
// reference's product nor its sum rounds); int -> double and the power-of-two
// scale are exact too.
__device__ __forceinline__ double pm1_of(uint32_t x) {
  return (double)(int)(2u * x - 0x80000000u) * 0x1p-31;
}

// The raw PCG32 XSH-RR output of state `old` (32 bits); rand() = raw >> 1.
__device__ __forceinline__ uint32_t pcg_raw32(uint64_t old) {
  const uint32_t xs = (uint32_t)(((old >> 18) ^ old) >> 27);
  const uint32_t rot = (uint32_t)(old >> 59);
  return (xs >> rot) | (xs << ((32u - rot) & 31u));
}

// rand31_x3 without the final >> 1 of each draw (see pm1_raw)
__device__ __forceinline__ void raw32_x3(uint64_t s0, uint32_t& r0, uint32_t& r1, uint32_t& r2,
                                         uint64_t& next) {
  const uint64_t s1 = s0 * 6364136223846793005ULL + 1442695040888963407ULL;
  const uint64_t s2 = s0 * 0x685f98a2018fade9ULL + 0x1a08ee1184ba6d32ULL;
  const uint64_t s3 = s0 * 0x0b046976f22528f5ULL + 0x9af678222e728119ULL;
  r0 = pcg_raw32(s0);
  r1 = pcg_raw32(s1);
  r2 = pcg_raw32(s2);
  next = s3;
}

// pm1_of(raw >> 1), from the raw 32-bit output: 2 (raw >> 1) = raw & ~1, and
// subtracting 2^31 mod 2^32 flips the top bit (one v_bitop3_b32).
__device__ __forceinline__ int pm1_int_raw(uint32_t raw) {
  return (int)((raw & 0xFFFFFFFEu) ^ 0x80000000u);
}
#ifndef PSRT_CVT_BIAS
#define PSRT_CVT_BIAS 1  // int -> double through the exponent bias (one FP64 add, no v_cvt)
#endif
// (double)pm1_int_raw(raw): with m = raw & ~1, the bits {hi 0x43300000, lo m}
// are the double 2^52 + m (exact), and (2^52 + m) - (2^52 + 2^31) = m - 2^31
// is exact (integers below 2^53, the difference below 2^31 in magnitude) and
// +0 when m = 2^31, as the conversion gives.
__device__ __forceinline__ double w_raw(uint32_t raw) {
#if PSRT_CVT_BIAS
  return __hiloint2double(0x43300000, (int)(raw & 0xFFFFFFFEu)) - 0x1.000008p52;
#else
  return (double)pm1_int_raw(raw);
#endif
}
__device__ __forceinline__ double pm1_raw(uint32_t raw) {
  return w_raw(raw) * 0x1p-31;
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

// random_in_unit_sphere's test (vec3.h:88): !(v.x*v.x + v.y*v.y + v.z*v.z > 1)
// on v = random(-1, 1) from raw draws (x, y, z), decided exactly in integers.
// With w = draw - 2^30, each coordinate is w * 2^-30 (pm1_of), so the exact
// sum is S * 2^-60, S = wx^2 + wy^2 + wz^2 < 3 * 2^60 (int64). The reference's
// FP64 sum (three rounded squares, two rounded adds) is within 2^-51 of it
// near 1, so when |S - 2^60| > 2^10 the integer comparison gives the same
// answer; in the band left (probability ~2^-49 per trial) the FP64 expression
// itself decides.
__device__ __forceinline__ bool in_unit_sphere(uint32_t x, uint32_t y, uint32_t z) {
  const int64_t wx = (int32_t)(x - 0x40000000u), wy = (int32_t)(y - 0x40000000u),
                wz = (int32_t)(z - 0x40000000u);
  const int64_t S = (wx * wx + wy * wy) + wz * wz;
  const int64_t dlt = S - (int64_t(1) << 60);
  if (dlt > 1024 || dlt < -1024) return dlt < 0 || dlt == 0;  // S <= 2^60
  const double rz = pm1_of(z), ry = pm1_of(y), rx = pm1_of(x);
  return !((rx * rx + ry * ry) + rz * rz > 1.0);
}

}  // namespace psrt
