/* psrt_trace's FP32 pre-decision of random_in_unit_sphere's test
 * (psrt_device.h in_unit_sphere_raw_f32; vec3.h:88 !(length_squared() > 1)
 * on raw rand() triples) against the FP64 test on the same triples, restated
 * in C: every triple the FP32 path decides must get the FP64 answer.
 * Random triples plus triples placed within 2^-18 of the sphere. Prints
 * "ok <decided> <undecided>" or the first mismatches. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>

static int32_t w_int(uint32_t raw) { return (int32_t)((raw & 0xFFFFFFFEu) ^ 0x80000000u); }
static int in64(uint32_t x, uint32_t y, uint32_t z) {
  const double wx = w_int(x), wy = w_int(y), wz = w_int(z);
  return !((wx * wx + wy * wy) + wz * wz > 0x1p62);
}
/* 1 inside, 0 outside, -1 undecided */
static int in32(uint32_t x, uint32_t y, uint32_t z) {
  const float fx = (float)w_int(x), fy = (float)w_int(y), fz = (float)w_int(z);
  const float s = fmaf(fx, fx, fmaf(fy, fy, fz * fz));
  if (s < 0x1p62f * (1.0f - 0x1p-20f)) return 1;
  if (s > 0x1p62f * (1.0f + 0x1p-20f)) return 0;
  return -1;
}
static uint64_t st = 0x9E3779B97F4A7C15ull;
static uint64_t next(void) {
  st ^= st << 13;
  st ^= st >> 7;
  st ^= st << 17;
  return st;
}
static uint32_t raw_of(double w) { /* raw whose w_int is the even integer nearest w */
  int64_t i = (int64_t)llround(w / 2.0) * 2;
  if (i > 2147483646) i = 2147483646;
  if (i < -2147483648LL) i = -2147483648LL;
  return ((uint32_t)(int32_t)i) ^ 0x80000000u;
}
int main(void) {
  long decided = 0, undecided = 0, bad = 0;
  for (long t = 0; t < 20000000; ++t) {
    uint32_t x, y, z;
    if (t & 1) {
      x = (uint32_t)next(), y = (uint32_t)next(), z = (uint32_t)next();
    } else { /* near the surface: a random direction scaled to radius 1 +- 2^-18 */
      double a = (double)(next() >> 11) * 0x1p-53 * 2 - 1, b = (double)(next() >> 11) * 0x1p-53 * 6.283185307179586;
      double rr = sqrt(1 - a * a), r = 1.0 + ((double)(next() >> 11) * 0x1p-53 * 2 - 1) * 0x1p-18;
      x = raw_of(0x1p31 * r * rr * cos(b)), y = raw_of(0x1p31 * r * rr * sin(b)), z = raw_of(0x1p31 * r * a);
    }
    const int f = in32(x, y, z);
    if (f < 0) {
      ++undecided;
      continue;
    }
    ++decided;
    if (f != in64(x, y, z)) {
      if (bad < 8) printf("mismatch %08x %08x %08x f32=%d f64=%d\n", x, y, z, f, in64(x, y, z));
      ++bad;
    }
  }
  if (bad) return 1;
  printf("ok %ld %ld\n", decided, undecided);
  return 0;
}
