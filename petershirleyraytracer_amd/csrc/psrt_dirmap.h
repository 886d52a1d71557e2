// psrt_dirmap.h — direction maps: exact "no BVH sphere ahead" proofs for rays
// that leave a sphere's surface.
//
// A ray that starts on sphere j (the previous hit) and that neither the hint
// test, the big spheres, the neighbour list nor the grid can bound used to
// walk the BVH — mostly rays escaping to the sky. A direction map answers it
// with one bit: for a patch P of j's surface and a bin B of directions, the
// bit is set when NO BVH sphere other than j can be met by any ray
// o + t d (t >= 0) with o within pad/2 of P and d in B. The hit record is
// then decided by the exact tests already done (j itself and the big
// spheres), as in the reference's scan (hittable_list.cc:9-17): every other
// sphere has no accepted root.
//
// Patches and direction bins are cells of the same cube map: face = the
// dominant axis of the vector and its sign; (s, t) = the other two
// coordinates (increasing axis order) divided by |dominant|; cell
// (i, j) = floor((s + 1) / 2 * M) clamped to [0, M). The device computes it in
// FP32 (error < 2^-21 in s, t); the host widens every cell by kDirEps on each
// side before bounding it, so the cell the device picks always covers the
// exact vector.
#pragma once

#include <cstdint>
#include <vector>

#include "psrt_bvh.h"

namespace psrt {

#ifndef PSRT_DIR_N
#define PSRT_DIR_N 8
#endif
constexpr int kDirN = PSRT_DIR_N;             // direction bins per cube-face edge
constexpr int kDirBins = 6 * kDirN * kDirN;   // bins per map
constexpr int kDirWords = kDirBins / 32;      // 32-bit words per map
static_assert(kDirBins % 64 == 0, "maps are written 64 bins per ballot");
constexpr double kDirEps = 0x1p-18;           // (s, t) widening of every cube cell
constexpr int kDirMaxM = 65535;               // patch cells per face edge (16-bit fields)

struct DirMapHost {
  // per (sphere, face), 4 ints: {first map or -1, M, i0 | j0 << 16, ni | nj << 16};
  // map of patch (i, j) (window-relative) = first + i * nj + j
  std::vector<int32_t> desc;
  std::vector<double> ball;     // per map: {mx, my, mz, rho}: origin region (a ball)
  std::vector<int32_t> excl;    // per map: the sphere the origin lies on (not a blocker), or -1
  std::vector<double> bins;     // per bin: {ax, ay, az, cos(ha), sin(ha), 0, 0, 0}
  int n_maps = 0;
  double h = 0.0;               // target patch edge (arc length)
};

// Plans the maps of a BVH scene: patches of every BVH sphere (whole surface)
// and of every big sphere (the part of its surface near the BVH spheres),
// their origin balls and the direction bins. Empty when the BVH is disabled
// or PSRT_NO_DIRMAP is set.
DirMapHost plan_dirmaps(const rt_sphere* s, int n, const BvhHost& b);

}  // namespace psrt
