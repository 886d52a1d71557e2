/* psrt_trace's div_by (psrt_kernels.hip): x / d for the camera ray's u and v
 * (main.cc:80-81, u = (i + random_double()) / (W - 1)) from y = RN(1/d) with
 * two FMA corrections, restated here in C (same operations, -ffp-contract=off)
 * and compared with IEEE division on every numerator form the kernel sees:
 * x = i + m 2^-31, 0 <= i < W, 0 <= m < 2^31 (random m plus the edge values).
 * Prints "ok <count>" or the first mismatches. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>

static double div_by(double x, double d, double y) {
  double q = x * y;
  double r = fma(-q, d, x);
  q = fma(r, y, q);
  r = fma(-q, d, x);
  return fma(r, y, q);
}

static uint64_t st = 88172645463325252ull;
static uint64_t next(void) {
  st ^= st << 13;
  st ^= st >> 7;
  st ^= st << 17;
  return st;
}

int main(void) {
  long bad = 0, tot = 0;
  for (int W = 2; W <= 20000; W += (W < 300 ? 1 : 37)) {
    const double d = W - 1, y = 1.0 / d;
    for (int t = 0; t < 4000; ++t) {
      const int i = (int)(next() % (uint64_t)W);
      uint32_t m = (uint32_t)(next() >> 33);
      if (t < 64) m = (t & 1) ? 0x7fffffffu - (t >> 1) : (uint32_t)(t >> 1);
      const double x = (t & 2) && t < 64 ? (double)(W - 1) + m * 0x1p-31 : (double)i + m * 0x1p-31;
      const double a = x / d, b = div_by(x, d, y);
      ++tot;
      if (a != b || signbit(a) != signbit(b)) {
        if (bad < 8) printf("W=%d x=%a ieee=%a div_by=%a\n", W, x, a, b);
        ++bad;
      }
    }
  }
  if (bad) return 1;
  printf("ok %ld\n", tot);
  return 0;
}
