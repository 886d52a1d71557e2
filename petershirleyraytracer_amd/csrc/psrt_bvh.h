// psrt_bvh.h — exact culling structure for hittable_list::hit.
//
// A binary BVH over the scene's "small" spheres, laid out depth-first with a
// skip link per node so the device walks it without a stack: on a box hit go
// to node+1 (first child), on a miss — or after a leaf — go to `skip`.
// "Big" spheres (radius > kBigRatio x the median radius, e.g. the r=1000
// ground) would bloat every box; they are tested on every ray instead.
//
// Boxes are the spheres' bounds padded by `pad` (absolute) and rounded
// outward to float. `pad` exceeds, with a wide margin, both the FP64 error of
// a computed root (the point o + t*d of any accepted root lies within ~1e-12
// of its sphere) and the FP32 slab-test error for ray origins with
// |o|_inf <= r_check; rays outside that range take the exact linear sweep.
#pragma once

#include <cstdint>
#include <vector>

#include "../../include/rt.h"

namespace psrt {

// 32 bytes: read as two float4 on the device.
struct BvhNode {
  float lo[3];
  int32_t skip;  // next node when this subtree is done/missed (== node count: end)
  float hi[3];
  int32_t leaf;  // -1 interior; else first << 8 | count (count <= 255)
};
static_assert(sizeof(BvhNode) == 32, "node layout");

constexpr int kBvhMinSpheres = 17;   // below this the linear sweep wins
constexpr double kBigRatio = 16.0;   // radius > 16 x median -> tested every ray
#ifndef PSRT_LEAF_MAX
#define PSRT_LEAF_MAX 2
#endif
#ifndef PSRT_LEAF_SAH_MAX
#define PSRT_LEAF_SAH_MAX 4  // SAH may stop splitting at this many spheres
#endif
#ifndef PSRT_SAH_AXES
#define PSRT_SAH_AXES 3  // binned SAH over the widest centroid axis (1) or all three (3)
#endif
#ifndef PSRT_SAH_YW
#define PSRT_SAH_YW 1.0  // SAH surface areas with the y extent scaled by this
#endif
#ifndef PSRT_TALL_RATIO
#define PSRT_TALL_RATIO 3.0  // > 0: spheres with r > this x median get their own root subtree
#endif
#ifndef PSRT_GRID_CELL
#define PSRT_GRID_CELL 2.5  // grid cell edge in median radii
#endif
constexpr int kLeafMax = PSRT_LEAF_MAX;
constexpr int kNbMax = 15;           // neighbour lists longer than this use the grid
constexpr int kListRecMax = 7;       // items of an inline grid-list record (BvhHost::cell_rec)
constexpr int kNbRecMax = 3;         // items of an inline neighbour record (BvhHost::nb_rec)
constexpr uint32_t kListOverflow = 0xFFFFu;

// Point-location grid over the same padded boxes: cell -> spheres whose padded
// box overlaps the cell. A ray whose segment [o, o + closest*d] lies inside one
// cell can only hit those spheres (its hit point is inside the hit sphere's
// padded box and inside the cell).
struct GridHost {
  // The device computes cell indices in FP32 from exactly these constants;
  // cell c on axis k spans [flo + c/finv, flo + (c+1)/finv] (exact reals).
  float flo[3] = {0, 0, 0};
  float fhi[3] = {0, 0, 0};  // >= flo + dims/finv: the grid's outer bound
  float finv = 1.0f;
  int dims[3] = {0, 0, 0};
  // 2 x ncell + 1 offsets into items (ncell = dims[0]*dims[1]*dims[2]): list
  // c < ncell is cell c; list ncell + c is the 2x2x2 block whose lowest cell
  // is c (union of up to 8 cell lists, deduplicated)
  std::vector<int32_t> start;
  std::vector<int32_t> items;  // original sphere indices
};

struct BvhHost {
  GridHost grid;
  std::vector<BvhNode> nodes;  // DFS order + one trailing padding node
  std::vector<int32_t> leaf_idx;  // original sphere index per leaf slot
  std::vector<int32_t> big_idx;   // original indices tested on every ray
  // Neighbour lists: for BVH sphere j, every BVH sphere k
  // with |c_j - c_k| <= |r_j| + |r_k| + 2 pad (k != j), i.e. every sphere whose
  // padded ball can meet j's. nb_word[j] = first << 4 | count (count <=
  // kNbMax); -1 for big spheres and spheres with more neighbours (grid path).
  std::vector<int32_t> nb_word;   // [n], by original index
  std::vector<int32_t> nb_items;  // original indices
  // The same lists as inline records, the form psrt_trace reads (one load per
  // query, no per-item loads): {count | i0 << 16, i1 | i2 << 16, ...} in
  // uint16 slots. cell_rec: 4 words per grid list (up to kListRecMax items);
  // nb_rec: 2 words per sphere (up to kNbRecMax). count = kListOverflow when
  // the list is longer, an index does not fit 16 bits, or (nb_rec) sphere j
  // has no neighbour list: the ray then takes the grid / the BVH walk.
  std::vector<uint32_t> cell_rec;  // [2 * ncell][4]
  std::vector<uint32_t> nb_rec;    // [n][2]
  double pad = 0.0;               // absolute box padding
  double r_check = 0.0;           // rays with |o|_inf > r_check use the linear sweep
  int depth = 0;
  bool enabled = false;
};

// Builds the structure; enabled = false when the scene is too small or
// degenerate (non-finite or non-positive radii, huge coordinates), in which
// case the device uses the linear sweep for every ray.
// big_ratio: radius ratio (to the median) above which a sphere is tested on
// every ray instead of entering the BVH; 0 = kBigRatio (rt_context_set_tuning)
BvhHost build_bvh(const rt_sphere* spheres, int n, double big_ratio = 0);

}  // namespace psrt
