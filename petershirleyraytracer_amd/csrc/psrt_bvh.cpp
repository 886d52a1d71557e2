// psrt_bvh.cpp — host build of the exact-culling BVH (see psrt_bvh.h).
#include "psrt_bvh.h"

#include <algorithm>
#include <cstdlib>
#include <cmath>
#include <limits>

namespace psrt {
namespace {

struct Box {
  double lo[3] = {std::numeric_limits<double>::infinity(), std::numeric_limits<double>::infinity(),
                  std::numeric_limits<double>::infinity()};
  double hi[3] = {-std::numeric_limits<double>::infinity(),
                  -std::numeric_limits<double>::infinity(),
                  -std::numeric_limits<double>::infinity()};
  void grow(const Box& b) {
    for (int k = 0; k < 3; ++k) {
      lo[k] = std::min(lo[k], b.lo[k]);
      hi[k] = std::max(hi[k], b.hi[k]);
    }
  }
  void grow(const double p[3]) {
    for (int k = 0; k < 3; ++k) {
      lo[k] = std::min(lo[k], p[k]);
      hi[k] = std::max(hi[k], p[k]);
    }
  }
  // surface area, the y extent weighted by PSRT_SAH_YW (1 = plain SAH)
  double area() const {
    const double dx = hi[0] - lo[0], dy = (hi[1] - lo[1]) * PSRT_SAH_YW, dz = hi[2] - lo[2];
    if (!(dx >= 0)) return 0.0;
    return 2.0 * (dx * dy + dy * dz + dz * dx);
  }
};

struct Prim {
  Box box;
  double c[3];
  int32_t idx;
};

// float rounding toward -inf / +inf of a double
float down(double x) {
  float f = (float)x;
  if ((double)f > x) f = std::nextafter(f, -std::numeric_limits<float>::infinity());
  return f;
}
float up(double x) {
  float f = (float)x;
  if ((double)f < x) f = std::nextafter(f, std::numeric_limits<float>::infinity());
  return f;
}

struct Builder {
  std::vector<Prim>& prims;
  BvhHost& out;

  // emit the subtree over prims[b, e) in DFS order; returns its node index
  int build(int b, int e, int depth) {
    out.depth = std::max(out.depth, depth);
    Box bounds, cbox;
    for (int i = b; i < e; ++i) {
      bounds.grow(prims[i].box);
      cbox.grow(prims[i].c);
    }
    const int me = (int)out.nodes.size();
    out.nodes.push_back(BvhNode{});
    BvhNode& nd0 = out.nodes[me];
    for (int k = 0; k < 3; ++k) {
      nd0.lo[k] = down(bounds.lo[k]);
      nd0.hi[k] = up(bounds.hi[k]);
    }
    const int count = e - b;
    int split = -1;
    if (count > kLeafMax) split = sah_split(b, e, cbox, bounds);
    if (split < 0) {
      out.nodes[me].leaf = ((int32_t)out.leaf_idx.size() << 8) | count;
      for (int i = b; i < e; ++i) out.leaf_idx.push_back(prims[i].idx);
    } else {
      out.nodes[me].leaf = -1;
      build(b, split, depth + 1);
      build(split, e, depth + 1);
    }
    out.nodes[me].skip = (int32_t)out.nodes.size();
    return me;
  }

  // root over prims[b, e) with the fixed children [b, m) and [m, e)
  int build_split_root(int b, int m, int e) {
    Box bounds;
    for (int i = b; i < e; ++i) bounds.grow(prims[i].box);
    const int me = (int)out.nodes.size();
    out.nodes.push_back(BvhNode{});
    for (int k = 0; k < 3; ++k) {
      out.nodes[me].lo[k] = down(bounds.lo[k]);
      out.nodes[me].hi[k] = up(bounds.hi[k]);
    }
    out.nodes[me].leaf = -1;
    build(b, m, 1);
    build(m, e, 1);
    out.nodes[me].skip = (int32_t)out.nodes.size();
    return me;
  }

  // binned SAH (PSRT_SAH_AXES 1: the widest centroid axis; 3: the best of
  // the three axes); -1 = make a leaf
  int sah_split(int b, int e, const Box& cbox, const Box& bounds) {
    int widest = 0;
    double wext = -1;
    for (int k = 0; k < 3; ++k)
      if (cbox.hi[k] - cbox.lo[k] > wext) wext = cbox.hi[k] - cbox.lo[k], widest = k;
    const int count = e - b;
    if (!(wext > 0)) {  // coincident centroids: split by count
      return count > 255 ? b + count / 2 : (count > kLeafMax ? b + count / 2 : -1);
    }
    constexpr int kBins = 16;
    double best = std::numeric_limits<double>::infinity();
    int best_k = -1, axis = widest;
    double ext = wext;
    for (int ax = 0; ax < 3; ++ax) {
      if (PSRT_SAH_AXES == 1 && ax != widest) continue;
      const double ex = cbox.hi[ax] - cbox.lo[ax];
      if (!(ex > 0)) continue;
      Box bb[kBins];
      int bc[kBins] = {0};
      for (int i = b; i < e; ++i) {
        const int k = std::min(kBins - 1, std::max(0, (int)((prims[i].c[ax] - cbox.lo[ax]) / ex * kBins)));
        bb[k].grow(prims[i].box);
        ++bc[k];
      }
      for (int k = 1; k < kBins; ++k) {
        Box l, r;
        int nl = 0, nr = 0;
        for (int j = 0; j < k; ++j)
          if (bc[j]) l.grow(bb[j]), nl += bc[j];
        for (int j = k; j < kBins; ++j)
          if (bc[j]) r.grow(bb[j]), nr += bc[j];
        if (!nl || !nr) continue;
        const double cost = l.area() * nl + r.area() * nr;
        if (cost < best) best = cost, best_k = k, axis = ax, ext = ex;
      }
    }
    auto bin_of = [&](const Prim& p) {
      int i = (int)((p.c[axis] - cbox.lo[axis]) / ext * kBins);
      return std::min(kBins - 1, std::max(0, i));
    };
    if (best_k < 0) return b + count / 2;  // all in one bin: split by count
    // cost model: traversal 1, intersection 2 (fp64 test ~ 2 fp32 box tests)
    const double leaf_cost = 2.0 * count;
    const double split_cost = 1.0 + 2.0 * best / std::max(bounds.area(), 1e-300);
    if (count <= PSRT_LEAF_SAH_MAX && leaf_cost <= split_cost) return -1;
    auto mid = std::partition(prims.begin() + b, prims.begin() + e,
                              [&](const Prim& p) { return bin_of(p) < best_k; });
    int m = (int)(mid - prims.begin());
    if (m == b || m == e) m = b + count / 2;
    return m;
  }
};

}  // namespace

BvhHost build_bvh(const rt_sphere* s, int n, double big_ratio_in) {
  BvhHost out;
  if (n < kBvhMinSpheres || !s) return out;
  std::vector<double> radii;
  radii.reserve(n);
  double scale = 0.0;
  for (int i = 0; i < n; ++i) {
    const double v[4] = {s[i].cx, s[i].cy, s[i].cz, s[i].r};
    for (double x : v)
      if (!std::isfinite(x) || std::fabs(x) > 1e6) return out;  // degenerate: linear sweep
    radii.push_back(std::fabs(s[i].r));
  }
  std::vector<double> sorted = radii;
  std::nth_element(sorted.begin(), sorted.begin() + n / 2, sorted.end());
  const double median = sorted[n / 2];
  const double big_ratio = big_ratio_in > 0 ? big_ratio_in : kBigRatio;  // Tuning::big_ratio
  std::vector<Prim> prims;
  for (int i = 0; i < n; ++i) {
    if (radii[i] > big_ratio * median && radii[i] > 0) {
      out.big_idx.push_back(i);
      continue;
    }
    const double c[3] = {s[i].cx, s[i].cy, s[i].cz};
    for (int k = 0; k < 3; ++k) scale = std::max(scale, std::fabs(c[k]) + radii[i]);
  }
  if ((int)out.big_idx.size() == n) return out;
  // pad = 2^-13 S (S = max |c| + r over the BVH spheres). Error budget
  // (DESIGN.md §8): the FP32 slab test's spatial error along an axis is
  // <= 2^-24 (5|o| + 4S) (origin and direction rounding, one subtract, one
  // multiply, the rounded-up tmax); the FP64 root error is ~1e-12. At
  // |o|_inf <= 64 S that is <= 2^-15.6 S, >6x inside the pad.
  scale = std::max(scale, 1.0);
  out.pad = std::ldexp(scale, -13);
  out.r_check = 64.0 * scale;
  for (int i = 0; i < n; ++i) {
    if (std::find(out.big_idx.begin(), out.big_idx.end(), i) != out.big_idx.end()) continue;
    Prim p;
    p.idx = i;
    p.c[0] = s[i].cx, p.c[1] = s[i].cy, p.c[2] = s[i].cz;
    for (int k = 0; k < 3; ++k) {
      p.box.lo[k] = p.c[k] - radii[i] - out.pad;
      p.box.hi[k] = p.c[k] + radii[i] + out.pad;
    }
    prims.push_back(p);
  }
  Builder bld{prims, out};
  // Tall spheres (radius > PSRT_TALL_RATIO x median, below the big class: the
  // final scene's three r = 1 spheres) get a subtree of their own under the
  // root. Otherwise their tall boxes top every subtree they share, and a
  // bounce ray leaving the sphere layer upward crosses those boxes for a long
  // stretch.
  const double tall = PSRT_TALL_RATIO * median;
  const auto mid = std::stable_partition(prims.begin(), prims.end(), [&](const Prim& p) {
    return !(tall > 0 && std::fabs(s[p.idx].r) > tall);
  });
  const int m = (int)(mid - prims.begin());
  if (m > 0 && m < (int)prims.size())
    bld.build_split_root(0, m, (int)prims.size());
  else
    bld.build(0, (int)prims.size(), 0);
  // padding node (never reached: the walk stops at nodes.size()); lets the
  // device read node+1 speculatively. Empty box, leaf word -1, skip = end.
  {
    BvhNode pad{};
    for (int k = 0; k < 3; ++k) pad.lo[k] = 1.0f, pad.hi[k] = -1.0f;
    pad.skip = (int32_t)out.nodes.size();
    pad.leaf = -1;
    out.nodes.push_back(pad);
  }

  // point-location grid: cells ~2.5 median radii wide, at most 128 per axis
  Box all;
  for (const Prim& p : prims) all.grow(p.box);
  double ext = 0.0;
  for (int k = 0; k < 3; ++k) ext = std::max(ext, all.hi[k] - all.lo[k]);
  double cell = std::max(PSRT_GRID_CELL * median, ext / 128.0);
  if (!(cell > 0)) cell = std::max(ext, 1.0);
  GridHost& g = out.grid;
  g.finv = (float)(1.0 / cell);
  const double inv = (double)g.finv;  // the cell size actually used: 1/finv
  long ncell = 1;
  for (int k = 0; k < 3; ++k) {
    g.flo[k] = down(all.lo[k]);
    g.dims[k] = std::max(1, (int)std::ceil((all.hi[k] - (double)g.flo[k]) * inv) + 1);
    g.fhi[k] = up((double)g.flo[k] + g.dims[k] / inv);
    ncell *= g.dims[k];
  }
  std::vector<std::vector<int32_t>> cells((size_t)ncell);
  auto cidx = [&](int x, int y, int z) { return ((long)z * g.dims[1] + y) * g.dims[0] + x; };
  // conservative membership: a sphere joins every cell its padded box touches,
  // boundaries included (the box is widened by 2^-30 of the scale first)
  const double eps = std::ldexp(scale, -30);
  for (const Prim& p : prims) {
    int c0[3], c1[3];
    for (int k = 0; k < 3; ++k) {
      const double a = std::floor((p.box.lo[k] - eps - (double)g.flo[k]) * inv);
      const double b = std::floor((p.box.hi[k] + eps - (double)g.flo[k]) * inv);
      c0[k] = (int)std::max(0.0, std::min((double)g.dims[k] - 1, a));
      c1[k] = (int)std::max(0.0, std::min((double)g.dims[k] - 1, b));
    }
    for (int z = c0[2]; z <= c1[2]; ++z)
      for (int y = c0[1]; y <= c1[1]; ++y)
        for (int x = c0[0]; x <= c1[0]; ++x) cells[cidx(x, y, z)].push_back(p.idx);
  }
  // lists [0, ncell): cells; [ncell, 2 ncell): 2x2x2 blocks, block b = the
  // union of cells (x..x+1, y..y+1, z..z+1) of cell b's corner (clipped to the
  // grid), for segments that cross at most one cell boundary per axis
  g.start.resize(2 * ncell + 1);
  g.start[0] = 0;
  for (long c = 0; c < ncell; ++c) {
    g.start[c + 1] = g.start[c] + (int32_t)cells[c].size();
    g.items.insert(g.items.end(), cells[c].begin(), cells[c].end());
  }
  std::vector<int32_t> blk;
  for (int z = 0; z < g.dims[2]; ++z)
    for (int y = 0; y < g.dims[1]; ++y)
      for (int x = 0; x < g.dims[0]; ++x) {
        blk.clear();
        for (int dz = 0; dz <= 1 && z + dz < g.dims[2]; ++dz)
          for (int dy = 0; dy <= 1 && y + dy < g.dims[1]; ++dy)
            for (int dx = 0; dx <= 1 && x + dx < g.dims[0]; ++dx) {
              const std::vector<int32_t>& cl = cells[cidx(x + dx, y + dy, z + dz)];
              blk.insert(blk.end(), cl.begin(), cl.end());
            }
        std::sort(blk.begin(), blk.end());
        blk.erase(std::unique(blk.begin(), blk.end()), blk.end());
        const long b = ncell + cidx(x, y, z);
        g.start[b + 1] = g.start[b] + (int32_t)blk.size();
        g.items.insert(g.items.end(), blk.begin(), blk.end());
      }

  // neighbour lists: two padded balls that meet have padded boxes that meet,
  // so both spheres share a cell (membership is conservative); candidates come
  // from the cells under j's box, the exact test is the centre distance
  out.nb_word.assign(n, -1);
  std::vector<int32_t> seen(n, -1), nb;
  for (const Prim& p : prims) {
    const int j = p.idx;
    int c0[3], c1[3];
    for (int k = 0; k < 3; ++k) {
      const double a = std::floor((p.box.lo[k] - eps - (double)g.flo[k]) * inv);
      const double b = std::floor((p.box.hi[k] + eps - (double)g.flo[k]) * inv);
      c0[k] = (int)std::max(0.0, std::min((double)g.dims[k] - 1, a));
      c1[k] = (int)std::max(0.0, std::min((double)g.dims[k] - 1, b));
    }
    nb.clear();
    bool many = false;
    for (int z = c0[2]; z <= c1[2] && !many; ++z)
      for (int y = c0[1]; y <= c1[1] && !many; ++y)
        for (int x = c0[0]; x <= c1[0] && !many; ++x) {
          const std::vector<int32_t>& cl = cells[cidx(x, y, z)];
          for (int32_t k : cl) {
            if (k == j || seen[k] == j) continue;
            seen[k] = j;
            const double dx = s[k].cx - s[j].cx, dy = s[k].cy - s[j].cy, dz = s[k].cz - s[j].cz;
            const double reach = (radii[j] + radii[k] + 2.0 * out.pad) * (1.0 + 0x1p-30);
            if (std::sqrt(dx * dx + dy * dy + dz * dz) <= reach) {
              nb.push_back(k);
              if ((int)nb.size() > kNbMax) {
                many = true;
                break;
              }
            }
          }
        }
    if (many) continue;
    std::sort(nb.begin(), nb.end());
    out.nb_word[j] = ((int32_t)out.nb_items.size() << 4) | (int32_t)nb.size();
    out.nb_items.insert(out.nb_items.end(), nb.begin(), nb.end());
  }

  // inline records (BvhHost::cell_rec / nb_rec): slot 0 the count, slots
  // 1.. the indices, in list order
  auto pack = [](const int32_t* it, int cnt, int cap, uint32_t* w, int words) {
    bool fits = cnt <= cap;
    for (int e = 0; e < cnt && fits; ++e) fits = it[e] >= 0 && it[e] < (int32_t)kListOverflow;
    uint16_t slot[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    slot[0] = fits ? (uint16_t)cnt : (uint16_t)kListOverflow;
    for (int e = 0; fits && e < cnt; ++e) slot[e + 1] = (uint16_t)it[e];
    for (int k = 0; k < words; ++k) w[k] = slot[2 * k] | (uint32_t)slot[2 * k + 1] << 16;
  };
  const size_t nlist = g.start.size() - 1;
  out.cell_rec.assign(4 * nlist, 0u);
  for (size_t c = 0; c < nlist; ++c)
    pack(g.items.data() + g.start[c], g.start[c + 1] - g.start[c], kListRecMax,
         &out.cell_rec[4 * c], 4);
  out.nb_rec.assign(2 * (size_t)n, 0u);
  for (int j = 0; j < n; ++j) {
    const int32_t w = out.nb_word[j];
    if (w < 0)
      pack(nullptr, kNbRecMax + 1, kNbRecMax, &out.nb_rec[2 * (size_t)j], 2);  // no list
    else
      pack(out.nb_items.data() + (w >> 4), w & 15, kNbRecMax, &out.nb_rec[2 * (size_t)j], 2);
  }
  out.enabled = true;
  return out;
}

}  // namespace psrt
