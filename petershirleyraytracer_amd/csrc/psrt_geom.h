// psrt_geom.h — FP64 / FP32 geometry primitives shared by the trace kernels
// (psrt_kernels.hip: the reference integrator; psrt_mat.hip: materials).
// Compiled with -ffp-contract=off, as psrt_device.h.
#pragma once

#include <hip/hip_runtime.h>

#include "psrt_kernels.h"

namespace psrt {

// sqrt (sphere.cc:19) as the compiler's correctly rounded f64 expansion
// (v_rsq_f64, then Goldschmidt/Newton steps), minus its range handling: for
// x >= 2^-767 the expansion's scaling is the identity and its zero / +inf
// fixup is not taken, so the steps below are exactly the ones it runs. Other
// inputs (0, tiny, +inf, NaN) take __builtin_sqrt behind a wave-uniform branch.
__device__ __forceinline__ double sqrt_f64(double x) {
  const double r = __builtin_amdgcn_rsq(x);
  double g = x * r;
  double h = r * 0.5;
  const double e = __builtin_fma(-h, g, 0.5);
  g = __builtin_fma(g, e, g);
  h = __builtin_fma(h, e, h);
  double d = __builtin_fma(-g, g, x);
  g = __builtin_fma(d, h, g);
  d = __builtin_fma(-g, g, x);
  g = __builtin_fma(d, h, g);
  const bool slow = !(x >= 0x1p-767 && x <= 0x1.fffffffffffffp1023);
  if (__builtin_expect(__ballot(slow) != 0, 0)) {
    if (slow) g = __builtin_sqrt(x);
  }
  return g;
}

// sphere.cc:34-36 + hittable.h:14-18 for the winning sphere:
// p = orig + dir*t (ray.h:25-28), outward = (p - c) / r = (1/r)*(p - c),
// front_face = dot(dir, outward) < 0, normal flipped to face the ray.
struct HitRec {
  double px, py, pz, nx, ny, nz;
  bool front;
};

__device__ __forceinline__ HitRec hit_record_of(const double4 s, double ir, double t, double ox,
                                                double oy, double oz, double dx, double dy,
                                                double dz) {
  HitRec h;
  h.px = ox + t * dx;
  h.py = oy + t * dy;
  h.pz = oz + t * dz;
  h.nx = ir * (h.px - s.x);
  h.ny = ir * (h.py - s.y);
  h.nz = ir * (h.pz - s.z);
  h.front = ((dx * h.nx + dy * h.ny) + dz * h.nz) < 0.0;
  if (!h.front) h.nx = -h.nx, h.ny = -h.ny, h.nz = -h.nz;
  return h;
}

__device__ __forceinline__ float tmax_up(double t) {
  // >= t for every finite t (float rounding <= 2^-24 relative; margin 2^-21)
  return (float)t * 1.00000048f;
}

__device__ __forceinline__ float safe_inv(float d) {
  const float m = __builtin_fabsf(d) < 1e-20f ? __builtin_copysignf(1e-20f, d) : d;
  return __builtin_amdgcn_rcpf(m);  // v_rcp_f32 (1 ulp): the padded boxes absorb it
}

// Conservative FP32 ray-box test over [tlo, tmax] (boxes padded, psrt_bvh.cpp)
// of a device node (psrt_kernels.h DevNode): n0 = {lo.x, lo.y, hi.x, hi.y},
// n1 = {lo.z, hi.z, skip, leaf}.
__device__ __forceinline__ bool slab_hit(const float4 n0, const float4 n1, float ix, float iy,
                                         float iz, float oix, float oiy, float oiz, float tlo,
                                         float tmax) {
  const float x0 = __builtin_fmaf(n0.x, ix, -oix), x1 = __builtin_fmaf(n0.z, ix, -oix);
  const float y0 = __builtin_fmaf(n0.y, iy, -oiy), y1 = __builtin_fmaf(n0.w, iy, -oiy);
  const float z0 = __builtin_fmaf(n1.x, iz, -oiz), z1 = __builtin_fmaf(n1.y, iz, -oiz);
  // v_min3/v_max3 directly: no NaN canonicalisation of tlo / tmax per box
  // (NaN cannot occur: finite boxes, safe_inv directions, finite tmax)
  float tn, tf, a, b;
  asm("v_min_f32 %0, %1, %2" : "=v"(a) : "v"(x0), "v"(x1));
  asm("v_min_f32 %0, %1, %2" : "=v"(b) : "v"(y0), "v"(y1));
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(tn) : "v"(a), "v"(b), "v"(tlo));
  asm("v_min_f32 %0, %1, %2" : "=v"(a) : "v"(z0), "v"(z1));
  asm("v_max_f32 %0, %1, %2" : "=v"(tn) : "v"(tn), "v"(a));
  asm("v_max_f32 %0, %1, %2" : "=v"(a) : "v"(x0), "v"(x1));
  asm("v_max_f32 %0, %1, %2" : "=v"(b) : "v"(y0), "v"(y1));
  asm("v_min3_f32 %0, %1, %2, %3" : "=v"(tf) : "v"(a), "v"(b), "v"(tmax));
  asm("v_max_f32 %0, %1, %2" : "=v"(a) : "v"(z0), "v"(z1));
  asm("v_min_f32 %0, %1, %2" : "=v"(tf) : "v"(tf), "v"(a));
  return tn <= tf;
}

// Entry t in [0, tmax] of the ray into the padded BVH root box, in FP64;
// negative if the segment misses the box.
__device__ __forceinline__ double root_box_entry(const BvhView& bv, double ox, double oy,
                                                 double oz, double dx, double dy, double dz,
                                                 double tmax) {
  const float4 ra = bv.nodes[0], rb = bv.nodes[1];
  double t0 = 0.0, t1 = tmax;
  const double o3[3] = {ox, oy, oz}, d3[3] = {dx, dy, dz};
  const double lo3[3] = {ra.x, ra.y, rb.x}, hi3[3] = {ra.z, ra.w, rb.y};  // DevNode layout
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    if (d3[k] == 0.0) {
      if (o3[k] < lo3[k] || o3[k] > hi3[k]) t0 = 2.0, t1 = 1.0;  // parallel, outside
    } else {
      const double inv = __builtin_amdgcn_rcp(d3[k]);  // v_rcp_f64; error << the pad
      const double u = (lo3[k] - o3[k]) * inv, v = (hi3[k] - o3[k]) * inv;
      t0 = __builtin_fmax(t0, __builtin_fmin(u, v));
      t1 = __builtin_fmin(t1, __builtin_fmax(u, v));
    }
  }
  return (t0 <= t1 * (1.0 + 0x1p-40) + 0x1p-40) ? t0 : -1.0;
}

// Point query for a short segment [o, o + bt*d] (the common case: the ray
// re-hit the sphere it starts on at t ~ 0). Returns the list (psrt_bvh.h
// GridHost: a cell, or the 2x2x2 block of cells the segment crosses into)
// whose spheres are the only BVH spheres the segment can hit, kGridOutside
// when the segment lies outside the grid (no BVH sphere can be hit), or
// kGridNone when it cannot be bounded this way (the BVH must be walked).
constexpr int kGridNone = -1, kGridOutside = -2;

// The uniform constants hit_quick / the walk read on every ray. psrt_trace
// keeps them in LDS and re-reads them per use (an LDS read issues on the LDS
// pipe); held in SGPRs across the loop they spill, and each reload from the
// spill lane is a VALU v_readlane (~20 per grid query).
struct GridC {
  float glo[3], ghi[3], ginv, gmargin;
  int gdims[3], ncell;
  // cell-index form of the widened segment bounds: fma(min, ginv, a0[k]) =
  // (min - m - glo) ginv and fma(max, ginv, a1[k]) = (max + m - glo) ginv, up
  // to FP32 rounding (~2^-24 of the coordinates, far inside the margin m)
  float a0[3], a1[3];
  int top[3], pad_;
  double r_check, nb_c2;
  const uint4* plist;  // BvhView::plist (psrt_trace's camera lists), or nullptr
};

__device__ __forceinline__ GridC grid_consts(const BvhView& bv) {
  GridC g;
  for (int k = 0; k < 3; ++k) {
    g.glo[k] = bv.glo[k], g.ghi[k] = bv.ghi[k], g.gdims[k] = bv.gdims[k];
    g.a0[k] = -(bv.glo[k] + bv.gmargin) * bv.ginv;
    g.a1[k] = -(bv.glo[k] - bv.gmargin) * bv.ginv;
    g.top[k] = bv.gdims[k] - 1;
  }
  g.ncell = bv.gdims[0] * bv.gdims[1] * bv.gdims[2];
  g.ginv = bv.ginv;
  g.gmargin = bv.gmargin;
  g.pad_ = 0;
  g.r_check = bv.r_check;
  g.nb_c2 = bv.nb_c2;
  g.plist = bv.plist;
  return g;
}


// floor(x) as int, saturating (NaN -> 0): one v_cvt_flr_i32_f32
__device__ __forceinline__ int cvt_flr_i32(float x) {
  int r;
  asm("v_cvt_flr_i32_f32 %0, %1" : "=v"(r) : "v"(x));
  return r;
}

// min(max(x, 0), hi): one v_med3_i32
__device__ __forceinline__ int clamp0_i32(int x, int hi) {
  int r;
  asm("v_med3_i32 %0, %1, 0, %2" : "=v"(r) : "v"(x), "v"(hi));
  return r;
}

__device__ __forceinline__ int grid_locate(const GridC& bv, double ox, double oy, double oz,
                                           double dx, double dy, double dz, double bt) {
  if (!(bt < 1e30)) return kGridNone;
  // FP32 is enough within the caller's range guard: the test is conservative
  // and its error is inside pad + margin (psrt_bvh.cpp, hit_quick)
  const float o3[3] = {(float)ox, (float)oy, (float)oz};
  const float d3[3] = {(float)dx, (float)dy, (float)dz};
  const float tb = (float)bt * 1.00000048f;
  int ci[3];
  bool outside = false, ok = true, one = true;
  // Cell range [c0, c1] of the widened segment per axis, from saturating
  // floor-converts (huge coordinates saturate, and the caller's range guard
  // keeps NaN out). Outside the grid when c1 < 0 or c0 > top on some axis:
  // the widened bound then lies below glo / at or past the grid's far side
  // (up to rounding far inside the margin), where no padded sphere box
  // reaches. Then clipped to the grid: a hit point lies in a padded sphere
  // box, hence in a cell of the grid.
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const float e = __builtin_fmaf(tb, d3[k], o3[k]);
    const int r0 = cvt_flr_i32(__builtin_fmaf(fminf(o3[k], e), bv.ginv, bv.a0[k]));
    const int r1 = cvt_flr_i32(__builtin_fmaf(fmaxf(o3[k], e), bv.ginv, bv.a1[k]));
    const int top = bv.top[k];
    outside = outside || r1 < 0 || r0 > top;
    const int c0 = clamp0_i32(r0, top), c1 = clamp0_i32(r1, top);
    ok = ok && c1 - c0 <= 1;
    one = one && c1 == c0;
    ci[k] = c0;
  }
  if (outside) return kGridOutside;
  if (!ok) return kGridNone;
  // one cell: its list; two cells on some axis: the 2x2x2 block list from ci
  const int cell = (ci[2] * bv.gdims[1] + ci[1]) * bv.gdims[0] + ci[0];
  return one ? cell : cell + bv.ncell;
}

}  // namespace psrt
