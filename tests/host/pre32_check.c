/* psrt_kernels.hip test_sphere's FP32 pre-reject (Pre32), checked against the
 * reference's own sphere test (sphere.cc:6-31 over [0, bt], FP64, -ffp-contract=off)
 * on adversarial cases: origins at distances 1e-13 .. 1e2 outside spheres of
 * radius 1e-3 .. 1e3 (the r = 1000 ground included), directions towards the
 * sphere, bt spread around D / |d|. Every rejected case must have no accepted
 * root; the device's v_sqrt_f32 (1 ulp) is modelled by rounding sqrt down 2 ulp.
 * The whole configuration is also scaled down by 2^-20 .. 2^-90 (ADVICE r04:
 * below ~2^-57 an absolute floor of 2^-100 in R let T*T lose its relative
 * accuracy; the floor is 2^-60, so T*T >= 2^-120 stays a normal float).
 * Prints "ok <cases> <rejected>" or the first violations.
 * -DR_FLOOR=0x1p-100 builds the old floor (it fails at the tiny scales). */
#include <math.h>
#include <stdint.h>
#include <stdio.h>

#ifndef R_FLOOR
#define R_FLOOR 0x1p-60 /* psrt_capi.hip pre32_sphere */
#endif

static uint64_t st = 0x9E3779B97F4A7C15ull;
static double u01(void) {
  st = st * 6364136223846793005ull + 1442695040888963407ull;
  return (double)(st >> 11) * 0x1p-53;
}

/* host R (psrt_capi.hip pre32_sphere) */
static float pre32_R(double cx, double cy, double cz, double r) {
  const double ar = fabs(r), cm = fmax(fabs(cx), fmax(fabs(cy), fabs(cz)));
  if (!(cm + ar <= 0x1p40)) return INFINITY;
  const double Rd = ar * (1.0 + 0x1p-18) + 0x1p-18 * cm + R_FLOOR;
  float R = (float)Rd;
  if ((double)R < Rd) R = nextafterf(R, INFINITY);
  return R;
}

static int reject32(double ox, double oy, double oz, double A, double am, double bt, double cx,
                    double cy, double cz, double r) {
  const float fox = (float)ox, foy = (float)oy, foz = (float)oz;
  const int ok = am <= 0x1p40 && A >= 0x1p-100 && A <= 0x1p100;
  float sq = sqrtf((float)A);
  sq = nextafterf(nextafterf(sq, 0.0f), 0.0f); /* device sqrt: up to 2 ulp low */
  const float sk = ok ? sq * (1.0f + 0x1p-16f) : INFINITY;
  const float mo = (float)am * (0x1p-18f * (1.0f + 0x1p-20f));
  const float R = pre32_R(cx, cy, cz, r);
  const float ax = fox - (float)cx, ay = foy - (float)cy, az = foz - (float)cz;
  const float L = fmaf(ax, ax, fmaf(ay, ay, az * az));
  const float T = fmaf((float)bt, sk, mo + R);
  return L > T * T;
}

/* sphere.cc:6-31 over [0, bt]: 1 if a root is accepted */
static int ref_hit(double ox, double oy, double oz, double dx, double dy, double dz, double cx,
                   double cy, double cz, double r, double bt) {
  const double ax = ox - cx, ay = oy - cy, az = oz - cz;
  const double A = dx * dx + dy * dy + dz * dz;
  const double hb = dx * ax + dy * ay + dz * az;
  const double C = ax * ax + ay * ay + az * az - r * r;
  const double disc = hb * hb - A * C;
  if (disc < 0) return 0;
  const double sq = sqrt(disc);
  double t = (-hb - sq) / A;
  if (t < 0 || t > bt) {
    t = (-hb + sq) / A;
    if (t < 0 || t > bt) return 0;
  }
  return 1;
}

int main(void) {
  long cases = 0, rej = 0, bad = 0;
  /* 4 M cases at scale 1, then 600 k at each smaller scale */
  static const double scales[] = {0x1p-20, 0x1p-40, 0x1p-57, 0x1p-64, 0x1p-70, 0x1p-80, 0x1p-90};
  const int n_scaled = 600000, n_plain = 4000000;
  for (int it = 0; it < n_plain + 7 * n_scaled; ++it) {
    const double S = it < n_plain ? 1.0 : scales[(it - n_plain) / n_scaled];
    double cx, cy, cz, r;
    const int kind = it % 4;
    if (kind == 0) {
      cx = 0, cy = -1000, cz = 0, r = 1000; /* the ground */
    } else {
      cx = (u01() - 0.5) * 40, cy = (u01() - 0.5) * 4, cz = (u01() - 0.5) * 40;
      r = pow(10.0, -3.0 + 4.0 * u01());
      if (it % 7 == 0) r = -r;
    }
    /* a point on the sphere, pushed out by D along the normal */
    double nx = u01() - 0.5, ny = u01() - 0.5, nz = u01() - 0.5;
    const double nl = sqrt(nx * nx + ny * ny + nz * nz);
    nx /= nl, ny /= nl, nz /= nl;
    const double D = pow(10.0, -13.0 + 15.0 * u01());
    cx *= S, cy *= S, cz *= S, r *= S;
    const double ar = fabs(r), Ds = D * S;
    const double ox = cx + nx * (ar + Ds), oy = cy + ny * (ar + Ds), oz = cz + nz * (ar + Ds);
    /* direction: towards the sphere (the centre, jittered), or random */
    double dx, dy, dz;
    if (it % 3) {
      dx = -nx + (u01() - 0.5) * 0.5, dy = -ny + (u01() - 0.5) * 0.5, dz = -nz + (u01() - 0.5) * 0.5;
    } else {
      dx = u01() - 0.5, dy = u01() - 0.5, dz = u01() - 0.5;
    }
    const double sc = pow(2.0, -4.0 + 8.0 * u01());
    dx *= sc, dy *= sc, dz *= sc;
    const double A = (dx * dx + dy * dy) + dz * dz;
    const double am = fmax(fabs(ox), fmax(fabs(oy), fabs(oz)));
    /* bt around D / |d|: 0, tiny, and D/|d| * (1 +- 2^-k) */
    const double base = Ds / sqrt(A);
    double bt;
    switch (it % 5) {
      case 0: bt = 0.0; break;
      case 1: bt = base * (1.0 - pow(2.0, -1.0 - 40.0 * u01())); break;
      case 2: bt = base * (1.0 + pow(2.0, -1.0 - 40.0 * u01())); break;
      case 3: bt = base * pow(10.0, -6.0 * u01()); break;
      default: bt = base * u01(); break;
    }
    ++cases;
    if (reject32(ox, oy, oz, A, am, bt, cx, cy, cz, r)) {
      ++rej;
      if (ref_hit(ox, oy, oz, dx, dy, dz, cx, cy, cz, r, bt)) {
        if (bad < 5)
          printf("violation: o=(%a,%a,%a) d=(%a,%a,%a) c=(%a,%a,%a) r=%a bt=%a\n", ox, oy, oz, dx,
                 dy, dz, cx, cy, cz, r, bt);
        ++bad;
      }
    }
  }
  if (bad) {
    printf("violations %ld\n", bad);
    return 1;
  }
  printf("ok %ld %ld\n", cases, rej);
  return 0;
}
