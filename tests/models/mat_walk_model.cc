// Walk-order model for the material kernel's batched walk: box tests per
// walked ray (bounce rays still unbounded after the big spheres) under the
// stackless skip-link DFS order (psrt_mat.hip hit_walk_m) and under a
// near-first order (children ordered by their box entry along the ray), and
// what a per-(sphere, direction bin) escape table would resolve (DESIGN.md §13,
// profiles/r05_matwalk). CPU only:
//   gcc -O2 -Ioracle -o /tmp/mat_rays tests/models/mat_walk_rays.c -lm && /tmp/mat_rays 20000 /tmp/mat_rays.bin
//   g++ -O2 -std=c++17 -Iinclude -Ipetershirleyraytracer_amd/csrc -o /tmp/mat_model tests/models/mat_walk_model.cc \
//       petershirleyraytracer_amd/csrc/psrt_bvh.cpp petershirleyraytracer_amd/csrc/psrt_scene.cpp && /tmp/mat_model /tmp/mat_rays.bin
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <vector>
#include "psrt_bvh.h"
extern "C" int rt_scene_book_final(unsigned seed, rt_sphere* out, rt_material* mats, int cap);
static bool sph_hit(const rt_sphere& s, const double o[3], const double d[3], double tmin, double tmax, double& t) {
  double ax = o[0]-s.cx, ay = o[1]-s.cy, az = o[2]-s.cz;
  double A = d[0]*d[0]+d[1]*d[1]+d[2]*d[2], hb = d[0]*ax+d[1]*ay+d[2]*az, C = ax*ax+ay*ay+az*az - s.r*s.r;
  double disc = hb*hb - A*C; if (disc < 0) return false;
  double sq = std::sqrt(disc); t = (-hb - sq)/A;
  if (t < tmin || t > tmax) { t = (-hb + sq)/A; if (t < tmin || t > tmax) return false; }
  return true;
}
static bool box(const psrt::BvhNode& nd, const double o[3], const double d[3], double tmax, double& te) {
  double t0 = 0, t1 = tmax;
  for (int k = 0; k < 3; ++k) {
    double inv = 1.0 / d[k];
    double u = (nd.lo[k] - o[k]) * inv, v = (nd.hi[k] - o[k]) * inv;
    if (u > v) std::swap(u, v);
    t0 = std::max(t0, u); t1 = std::min(t1, v);
  }
  te = t0; return t0 <= t1;
}
int main(int argc, char** argv) {
  std::vector<rt_sphere> sph(600); std::vector<rt_material> mats(600);
  int n = rt_scene_book_final(1, sph.data(), mats.data(), 600); sph.resize(n);
  psrt::BvhHost b = psrt::build_bvh(sph.data(), n);
  const int m = (int)b.nodes.size() - 1;
  int walk0 = (m > 1 && b.nodes[0].leaf < 0) ? 1 : 0;
  const int N = 8, NB = 6*N*N;
  auto bin_of = [&](const double d[3]) {
    double a[3] = {std::fabs(d[0]), std::fabs(d[1]), std::fabs(d[2])};
    int f = (a[0] >= a[1] && a[0] >= a[2]) ? 0 : (a[1] >= a[2] ? 1 : 2);
    int u = f == 0 ? 1 : 0, v = f == 2 ? 1 : 2;
    int i = std::min(N-1, std::max(0, (int)std::floor((d[u]/a[f] + 1) * 0.5 * N)));
    int jj = std::min(N-1, std::max(0, (int)std::floor((d[v]/a[f] + 1) * 0.5 * N)));
    return ((2*f + (d[f] < 0)) * N + jj) * N + i;
  };
  std::vector<int> memo((size_t)n * NB, -1);
  auto esc_empty = [&](int j, int bb) {
    int& r = memo[(size_t)j * NB + bb];
    if (r >= 0) return r == 1;
    int face = bb / (N*N), cj = (bb / N) % N, ci = bb % N, f = face >> 1;
    int u = f == 0 ? 1 : 0, v = f == 2 ? 1 : 2; double sg = (face & 1) ? -1 : 1;
    auto dir = [&](double s, double t, double out[3]) { out[f] = sg; out[u] = s; out[v] = t;
      double l = std::sqrt(out[0]*out[0]+out[1]*out[1]+out[2]*out[2]); for (int q=0;q<3;++q) out[q]/=l; };
    double st = 2.0/N, s0 = -1+ci*st, t0 = -1+cj*st, ax[3], dd[3];
    dir(s0+st/2, t0+st/2, ax); double cmin = 1;
    for (int e=0;e<4;++e){ dir(e&1? s0+st:s0, e>>1? t0+st:t0, dd); cmin = std::min(cmin, ax[0]*dd[0]+ax[1]*dd[1]+ax[2]*dd[2]); }
    double ca = cmin - 1e-5, sa = std::sqrt(std::max(0.0, 1-ca*ca));
    bool empty = true;
    for (int k : b.leaf_idx) {
      if (k == j) continue;
      double cx = sph[k].cx-sph[j].cx, cy = sph[k].cy-sph[j].cy, cz = sph[k].cz-sph[j].cz;
      double l = std::sqrt(cx*cx+cy*cy+cz*cz);
      double R = std::fabs(sph[j].r) + std::fabs(sph[k].r) + 2*b.pad;
      if (l <= R + b.pad) continue;  // neighbour: tested exactly (its list)
      R = std::fabs(sph[j].r) + std::fabs(sph[k].r) + 1.5*b.pad;
      double cb = (ax[0]*cx+ax[1]*cy+ax[2]*cz)/l;
      if (cb >= ca) { empty = false; break; }
      double sb = std::sqrt(std::max(0.0, 1-cb*cb)), cosd = cb*ca+sb*sa, sind = sb*ca-cb*sa;
      if (cosd >= 0 && sind <= R/l) { empty = false; break; }
    }
    r = empty ? 1 : 0; return empty;
  };
  long from_sphere = 0, ground_or_other = 0, caught = 0; double cbox = 0, gbox = 0;
  FILE* f = fopen(argc > 1 ? argv[1] : "mat_rays.bin", "rb");
  if (!f) return 1;
  double w[9];
  long walked = 0, hits = 0; double box1 = 0, box2 = 0, box2h = 0, box1h = 0, sp1 = 0, sp2 = 0;
  while (fread(w, sizeof w, 1, f) == 1) {
    if (w[8] < 1) continue;  // camera rays: lens lists
    const double o[3] = {w[0], w[1], w[2]}, d[3] = {w[3], w[4], w[5]};
    double bt = INFINITY, t; int bi = -1;
    for (int q : b.big_idx) if (sph_hit(sph[q], o, d, 0.001, bt, t)) { bt = t; bi = q; }
    if (bt < INFINITY) continue;  // bounded: the grid decides most
    ++walked;
    // (1) skip-link DFS from walk0
    double bt1 = bt; int bi1 = bi; long c1 = 0, s1 = 0;
    for (int node = walk0; node < m;) {
      const psrt::BvhNode& nd = b.nodes[node]; double te; ++c1;
      if (!box(nd, o, d, bt1, te)) { node = nd.skip; continue; }
      if (nd.leaf >= 0) {
        for (int e = (nd.leaf >> 8); e < (nd.leaf >> 8) + (nd.leaf & 255); ++e) {
          int k = b.leaf_idx[e]; ++s1;
          if (sph_hit(sph[k], o, d, 0.001, bt1, t) && (t < bt1 || k > bi1)) { bt1 = t; bi1 = k; }
        }
        node = nd.skip;
      } else node = node + 1;
    }
    // (2) near-first with a stack: expand a node by testing its children's boxes
    double bt2 = bt; int bi2 = bi; long c2 = 0, s2 = 0;
    std::vector<std::pair<double,int>> st; st.push_back({0.0, 0});
    while (!st.empty()) {
      auto [te0, node] = st.back(); st.pop_back();
      if (te0 > bt2) continue;
      const psrt::BvhNode& nd = b.nodes[node];
      if (nd.leaf >= 0) {
        for (int e = (nd.leaf >> 8); e < (nd.leaf >> 8) + (nd.leaf & 255); ++e) {
          int k = b.leaf_idx[e]; ++s2;
          if (sph_hit(sph[k], o, d, 0.001, bt2, t) && (t < bt2 || k > bi2)) { bt2 = t; bi2 = k; }
        }
        continue;
      }
      std::vector<std::pair<double,int>> kids;
      for (int ch = node + 1; ch < nd.skip; ch = b.nodes[ch].skip) {
        double te; ++c2;
        if (box(b.nodes[ch], o, d, bt2, te)) kids.push_back({te, ch});
      }
      std::sort(kids.begin(), kids.end(), [](auto& x, auto& y){ return x.first > y.first; });
      for (auto& k : kids) st.push_back(k);
    }
    if (bi1 != bi2) { printf("MISMATCH\n"); return 1; }
    // escape table: origin on a BVH sphere j (|C| small), table bit of (j, bin(d))
    {
      int j = -1;
      for (int k : b.leaf_idx) {
        double ax=o[0]-sph[k].cx, ay=o[1]-sph[k].cy, az=o[2]-sph[k].cz;
        double C = ax*ax+ay*ay+az*az - sph[k].r*sph[k].r;
        if (std::fabs(C) <= 0.25*b.pad*std::fabs(sph[k].r)) { j = k; break; }
      }
      if (j < 0) { ++ground_or_other; gbox += c1; }
      else {
        ++from_sphere;
        if (esc_empty(j, bin_of(d))) { ++caught; cbox += c1; }
      }
    }
    box1 += c1; box2 += c2; sp1 += s1; sp2 += s2;
    if (bi1 >= 0) { ++hits; box1h += c1; box2h += c2; }
  }
  printf("walked %ld (hit %ld): boxes/ray skip-DFS %.2f near-first %.2f; on hitting rays %.2f vs %.2f; "
         "sphere tests/ray %.2f vs %.2f\n", walked, hits, box1/walked, box2/walked,
         box1h/std::max(1L,hits), box2h/std::max(1L,hits), sp1/walked, sp2/walked);
  printf("walked from BVH spheres %ld, from the ground/other %ld (their boxes %.0f%%); escape table N=%d "
         "catches %ld = %.1f%% of walked rays, %.1f%% of walked box tests\n", from_sphere, ground_or_other,
         100*gbox/box1, N, caught, 100.0*caught/walked, 100*cbox/box1);
}
