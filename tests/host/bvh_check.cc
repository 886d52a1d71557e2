// Invariants of the exact-culling structures (psrt_bvh.cpp), checked on CPU.
// Prints "ok <nodes> <big> <cells> <items>" or "FAIL <what>".
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "../../petershirleyraytracer_amd/csrc/psrt_bvh.h"

static int fails = 0;
#define CHECK(c, what)                     \
  do {                                     \
    if (!(c)) {                            \
      std::printf("FAIL %s\n", what);      \
      ++fails;                             \
      return;                              \
    }                                      \
  } while (0)

static void check_scene(const std::vector<rt_sphere>& s) {
  const psrt::BvhHost b = psrt::build_bvh(s.data(), (int)s.size());
  if (!b.enabled) {
    std::printf("disabled %zu\n", s.size());
    return;
  }
  const int n = (int)s.size();
  std::vector<int> seen(n, 0);
  for (int i : b.big_idx) seen[i] += 1;
  for (int i : b.leaf_idx) seen[i] += 1;
  for (int i = 0; i < n; ++i) CHECK(seen[i] == 1, "every sphere in exactly one leaf or the big list");
  const int m = (int)b.nodes.size() - 1;  // last node is padding
  CHECK(b.nodes[m].leaf == -1 && b.nodes[m].lo[0] > b.nodes[m].hi[0], "padding node is empty");
  CHECK(b.nodes[0].skip == m, "root skip == end");
  // walk: every node's subtree is [k+1, skip); leaves own slots; boxes nest
  for (int k = 0; k < m; ++k) {
    const psrt::BvhNode& nd = b.nodes[k];
    CHECK(nd.skip > k && nd.skip <= m, "skip link in range");
    for (int a = 0; a < 3; ++a) CHECK(nd.lo[a] <= nd.hi[a], "box ordered");
    if (nd.leaf >= 0) {
      CHECK(nd.skip == k + 1, "leaf has no children");
      const int first = nd.leaf >> 8, cnt = nd.leaf & 255;
      CHECK(cnt >= 1 && first + cnt <= (int)b.leaf_idx.size(), "leaf range");
      for (int e = first; e < first + cnt; ++e) {
        const rt_sphere& sp = s[b.leaf_idx[e]];
        const double c[3] = {sp.cx, sp.cy, sp.cz}, r = std::fabs(sp.r);
        for (int a = 0; a < 3; ++a) {
          CHECK((double)nd.lo[a] <= c[a] - r - b.pad, "leaf box holds padded sphere (lo)");
          CHECK((double)nd.hi[a] >= c[a] + r + b.pad, "leaf box holds padded sphere (hi)");
        }
      }
    } else {
      CHECK(nd.skip > k + 1, "interior has children");
      // children: k+1 and then skip of k+1, ... until nd.skip
      int ch = k + 1, kids = 0;
      while (ch < nd.skip) {
        const psrt::BvhNode& c = b.nodes[ch];
        for (int a = 0; a < 3; ++a) CHECK(nd.lo[a] <= c.lo[a] && nd.hi[a] >= c.hi[a], "boxes nest");
        ch = c.skip;
        ++kids;
      }
      CHECK(ch == nd.skip && kids == 2, "binary node with contiguous subtrees");
    }
  }
  // grid: each BVH sphere listed in every cell its padded box touches
  const psrt::GridHost& g = b.grid;
  const double inv = (double)g.finv;
  for (int e = 0; e < (int)b.leaf_idx.size(); ++e) {
    const int i = b.leaf_idx[e];
    const double c[3] = {s[i].cx, s[i].cy, s[i].cz}, r = std::fabs(s[i].r) + b.pad;
    int lo[3], hi[3];
    for (int a = 0; a < 3; ++a) {
      CHECK((double)g.flo[a] <= c[a] - r && (double)g.fhi[a] >= c[a] + r, "grid bounds hold box");
      lo[a] = (int)std::floor((c[a] - r - (double)g.flo[a]) * inv);
      hi[a] = (int)std::floor((c[a] + r - (double)g.flo[a]) * inv);
      lo[a] = std::max(0, lo[a]);
      hi[a] = std::min(g.dims[a] - 1, hi[a]);
    }
    for (int z = lo[2]; z <= hi[2]; ++z)
      for (int y = lo[1]; y <= hi[1]; ++y)
        for (int x = lo[0]; x <= hi[0]; ++x) {
          const long cell = ((long)z * g.dims[1] + y) * g.dims[0] + x;
          bool found = false;
          for (int t = g.start[cell]; t < g.start[cell + 1]; ++t) found |= g.items[t] == i;
          CHECK(found, "sphere listed in every touched cell");
        }
  }
  // 2x2x2 block lists: list ncell + c = the deduplicated union of the cell
  // lists of the (clipped) block whose lowest cell is c
  const long ncell = (long)g.dims[0] * g.dims[1] * g.dims[2];
  CHECK((long)g.start.size() == 2 * ncell + 1, "cell lists then block lists");
  for (int z = 0; z < g.dims[2]; ++z)
    for (int y = 0; y < g.dims[1]; ++y)
      for (int x = 0; x < g.dims[0]; ++x) {
        std::vector<int> want;
        for (int dz = 0; dz <= 1 && z + dz < g.dims[2]; ++dz)
          for (int dy = 0; dy <= 1 && y + dy < g.dims[1]; ++dy)
            for (int dx = 0; dx <= 1 && x + dx < g.dims[0]; ++dx) {
              const long cell = ((long)(z + dz) * g.dims[1] + y + dy) * g.dims[0] + x + dx;
              for (int t = g.start[cell]; t < g.start[cell + 1]; ++t) want.push_back(g.items[t]);
            }
        std::sort(want.begin(), want.end());
        want.erase(std::unique(want.begin(), want.end()), want.end());
        const long bl = ncell + ((long)z * g.dims[1] + y) * g.dims[0] + x;
        const std::vector<int> got(g.items.begin() + g.start[bl], g.items.begin() + g.start[bl + 1]);
        CHECK(got == want, "block list = union of its cells");
      }
  // neighbour lists: exactly the BVH spheres within |r_j| + |r_k| + 2 pad, or -1
  std::vector<char> big(n, 0);
  for (int i : b.big_idx) big[i] = 1;
  CHECK((int)b.nb_word.size() == n, "one neighbour word per sphere");
  for (int j = 0; j < n; ++j) {
    if (big[j]) {
      CHECK(b.nb_word[j] == -1, "big spheres use the grid path");
      continue;
    }
    std::vector<int> want;
    for (int k = 0; k < n; ++k) {
      if (k == j || big[k]) continue;
      const double dx = s[k].cx - s[j].cx, dy = s[k].cy - s[j].cy, dz = s[k].cz - s[j].cz;
      const double reach = (std::fabs(s[j].r) + std::fabs(s[k].r) + 2.0 * b.pad) * (1.0 + 0x1p-30);
      if (std::sqrt(dx * dx + dy * dy + dz * dz) <= reach) want.push_back(k);
    }
    const int w = b.nb_word[j];
    if ((int)want.size() > psrt::kNbMax) {
      CHECK(w == -1, "long neighbour lists fall back to the grid");
      continue;
    }
    CHECK(w >= 0 && (w & 15) == (int)want.size(), "neighbour count");
    for (int e = 0; e < (int)want.size(); ++e)
      CHECK(b.nb_items[(w >> 4) + e] == want[e], "neighbour list = all spheres in reach, sorted");
  }
  // inline records (what psrt_trace reads): slot 0 the count, then the list
  // in order; kListOverflow exactly when the list does not fit
  auto slots = [](const uint32_t* w, int words, int k) { return (int)((w[k / 2] >> (16 * (k % 2))) & 0xFFFFu); };
  CHECK(b.cell_rec.size() == 4 * (g.start.size() - 1), "one record per grid list");
  for (size_t c = 0; c + 1 < g.start.size(); ++c) {
    const int cnt = g.start[c + 1] - g.start[c];
    const uint32_t* w = &b.cell_rec[4 * c];
    if (cnt > psrt::kListRecMax) {
      CHECK(slots(w, 4, 0) == (int)psrt::kListOverflow, "long grid lists overflow their record");
      continue;
    }
    CHECK(slots(w, 4, 0) == cnt, "grid record count");
    for (int e = 0; e < cnt; ++e) CHECK(slots(w, 4, e + 1) == g.items[g.start[c] + e], "grid record items");
  }
  CHECK(b.nb_rec.size() == 2 * (size_t)n, "one neighbour record per sphere");
  for (int j = 0; j < n; ++j) {
    const int w = b.nb_word[j];
    const uint32_t* r = &b.nb_rec[2 * (size_t)j];
    if (w < 0 || (w & 15) > psrt::kNbRecMax) {
      CHECK(slots(r, 2, 0) == (int)psrt::kListOverflow, "neighbour record overflow = grid path");
      continue;
    }
    CHECK(slots(r, 2, 0) == (w & 15), "neighbour record count");
    for (int e = 0; e < (w & 15); ++e) CHECK(slots(r, 2, e + 1) == b.nb_items[(w >> 4) + e], "neighbour record items");
  }
  std::printf("ok %d %zu %zu %zu\n", m, b.big_idx.size(), ncell, g.items.size());
}

int main() {
  std::vector<rt_sphere> fin((size_t)1024);
  const int nf = rt_scene_random_spheres(1, fin.data(), 1024);
  fin.resize(nf);
  check_scene(fin);
  std::mt19937_64 rng(7);
  std::uniform_real_distribution<double> U(-5, 5), R(0.01, 0.7);
  for (int t = 0; t < 6; ++t) {
    std::vector<rt_sphere> s;
    const int n = 20 + t * 300;
    for (int i = 0; i < n; ++i) s.push_back({U(rng), U(rng), U(rng), (t % 2 ? -1 : 1) * R(rng)});
    if (t >= 3) s.push_back({0, -1000, 0, 1000});
    if (t == 5) s.insert(s.end(), s.begin(), s.begin() + 50);  // duplicates
    check_scene(s);
  }
  std::vector<rt_sphere> coinc(40, rt_sphere{0, 0, 0, 1});
  check_scene(coinc);
  std::vector<rt_sphere> small(5, rt_sphere{0, 0, 0, 1});
  check_scene(small);
  return fails ? 1 : 0;
}
