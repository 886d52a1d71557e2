/* psrt_device.h pm1_raw, checked on every even 32-bit raw draw (the odd ones
 * give the same m = raw & ~1): the one-add form {hi 0x41400000, lo m} -
 * (2^21 + 1) against random_double(-1, 1) of the draw rand() = raw >> 1
 * (random.h:10-14: -1 + 2 * (rand() / 2^31)) and against the r03 two-op form.
 * Prints "ok <count>" or the first mismatches. */
#include <stdint.h>
#include <stdio.h>
#include <string.h>

static double hilo(uint32_t hi, uint32_t lo) {
  const uint64_t b = ((uint64_t)hi << 32) | lo;
  double d;
  memcpy(&d, &b, 8);
  return d;
}

int main(void) {
  uint64_t bad = 0, n = 0;
  for (uint64_t r = 0; r < (1ull << 32); r += 2, ++n) {
    const uint32_t raw = (uint32_t)r;
    const double ref = -1.0 + 2.0 * ((double)(raw >> 1) / 2147483648.0);
    const double old = (hilo(0x43300000u, raw & 0xFFFFFFFEu) - 0x1.000008p52) * 0x1p-31;
    const double now = hilo(0x41400000u, raw & 0xFFFFFFFEu) - 0x1.000008p21;
    uint64_t a, b, c;
    memcpy(&a, &ref, 8);
    memcpy(&b, &old, 8);
    memcpy(&c, &now, 8);
    if (a != b || a != c) {
      if (bad < 5) printf("mismatch raw=%u %a %a %a\n", raw, ref, old, now);
      ++bad;
    }
  }
  if (bad) return 1;
  printf("ok %llu\n", (unsigned long long)n);
  return 0;
}
