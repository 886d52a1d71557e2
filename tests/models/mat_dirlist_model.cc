// Direction-list model for the material kernel (r05): the rays the batched
// walk takes (bounce rays the big spheres leave unbounded) start on a surface
// the previous bounce hit: the ground (a big sphere) or a BVH sphere j. Per
// (origin patch, cube-map direction bin) a list of every BVH sphere a ray from
// that patch in that bin can meet (padded ball against the bin's cone from the
// patch, widened by the patch's radius) would decide such a ray with a few
// exact tests, as the camera-ray lists do, when the list is
// short. Patches: a square grid of cells (edge g) on the ground; sphere j
// itself for BVH origins (apex c_j, balls widened by |r_j|, j always listed).
// Reports the share of walked rays and of their box tests such lists resolve,
// and checks that every ray's true closest hit is listed. CPU only:
//   gcc -O2 -Ioracle -o /tmp/mat_rays tests/models/mat_walk_rays.c -lm && /tmp/mat_rays 20000 /tmp/mat_rays.bin
//   g++ -O2 -std=c++17 -Iinclude -Ipetershirleyraytracer_amd/csrc -o /tmp/mat_dl tests/models/mat_dirlist_model.cc \
//       petershirleyraytracer_amd/csrc/psrt_bvh.cpp petershirleyraytracer_amd/csrc/psrt_scene.cpp && /tmp/mat_dl /tmp/mat_rays.bin 8 0.5
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <vector>
#include "psrt_bvh.h"
extern "C" int rt_scene_book_final(unsigned seed, rt_sphere* out, rt_material* mats, int cap);

static bool sph_hit(const rt_sphere& s, const double o[3], const double d[3], double tmin, double tmax,
                    double& t) {
  double ax = o[0] - s.cx, ay = o[1] - s.cy, az = o[2] - s.cz;
  double A = d[0] * d[0] + d[1] * d[1] + d[2] * d[2], hb = d[0] * ax + d[1] * ay + d[2] * az;
  double C = ax * ax + ay * ay + az * az - s.r * s.r;
  double disc = hb * hb - A * C;
  if (disc < 0) return false;
  double sq = std::sqrt(disc);
  t = (-hb - sq) / A;
  if (t < tmin || t > tmax) {
    t = (-hb + sq) / A;
    if (t < tmin || t > tmax) return false;
  }
  return true;
}
static bool box(const psrt::BvhNode& nd, const double o[3], const double d[3], double tmax) {
  double t0 = 0, t1 = tmax;
  for (int k = 0; k < 3; ++k) {
    double inv = 1.0 / d[k];
    double u = (nd.lo[k] - o[k]) * inv, v = (nd.hi[k] - o[k]) * inv;
    if (u > v) std::swap(u, v);
    t0 = std::max(t0, u);
    t1 = std::min(t1, v);
  }
  return t0 <= t1;
}

int main(int argc, char** argv) {
  const char* path = argc > 1 ? argv[1] : "mat_rays.bin";
  const int N = argc > 2 ? atoi(argv[2]) : 8;
  const double g = argc > 3 ? atof(argv[3]) : 0.5;
  const int kMax = 7;
  const bool cellmode = argc > 4 && argv[4][0] == 'c';  // "cell": 3-D cells keyed for every origin
  std::vector<rt_sphere> sph(600);
  std::vector<rt_material> mats(600);
  int n = rt_scene_book_final(1, sph.data(), mats.data(), 600);
  sph.resize(n);
  psrt::BvhHost b = psrt::build_bvh(sph.data(), n);
  const int m = (int)b.nodes.size() - 1;
  const int walk0 = (m > 1 && b.nodes[0].leaf < 0) ? 1 : 0;
  const int ground = b.big_idx.empty() ? -1 : b.big_idx[0];
  // cube-map bins: axis and cos / sin of the half-angle to the corners
  const int NB = 6 * N * N;
  std::vector<double> ax(3 * NB), ca(NB), sa(NB);
  for (int bb = 0; bb < NB; ++bb) {
    int face = bb / (N * N), cj = (bb / N) % N, ci = bb % N, f = face >> 1;
    int u = f == 0 ? 1 : 0, v = f == 2 ? 1 : 2;
    double sg = (face & 1) ? -1 : 1;
    auto dir = [&](double s, double t, double out[3]) {
      out[f] = sg, out[u] = s, out[v] = t;
      double l = std::sqrt(out[0] * out[0] + out[1] * out[1] + out[2] * out[2]);
      for (int q = 0; q < 3; ++q) out[q] /= l;
    };
    double st = 2.0 / N, s0 = -1 + ci * st, t0 = -1 + cj * st, a[3], dd[3];
    dir(s0 + st / 2, t0 + st / 2, a);
    double cmin = 1;
    for (int e = 0; e < 4; ++e) {
      dir(e & 1 ? s0 + st : s0, e >> 1 ? t0 + st : t0, dd);
      cmin = std::min(cmin, a[0] * dd[0] + a[1] * dd[1] + a[2] * dd[2]);
    }
    double ang = std::acos(std::max(-1.0, std::min(1.0, cmin))) + 1e-6;
    for (int q = 0; q < 3; ++q) ax[3 * bb + q] = a[q];
    ca[bb] = std::cos(ang), sa[bb] = std::sin(ang);
  }
  auto bin_of = [&](const double d[3]) {
    double a[3] = {std::fabs(d[0]), std::fabs(d[1]), std::fabs(d[2])};
    int f = (a[0] >= a[1] && a[0] >= a[2]) ? 0 : (a[1] >= a[2] ? 1 : 2);
    int u = f == 0 ? 1 : 0, v = f == 2 ? 1 : 2;
    int i = std::min(N - 1, std::max(0, (int)std::floor((d[u] / a[f] + 1) * 0.5 * N)));
    int jj = std::min(N - 1, std::max(0, (int)std::floor((d[v] / a[f] + 1) * 0.5 * N)));
    return ((2 * f + (d[f] < 0)) * N + jj) * N + i;
  };
  // does the cone (apex p, bin bb) meet ball(c, R)?
  auto meets = [&](int bb, const double p[3], const rt_sphere& s, double R) {
    double w[3] = {s.cx - p[0], s.cy - p[1], s.cz - p[2]};
    double l = std::sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
    if (l <= R * (1 + 1e-9)) return true;
    double cb = (ax[3 * bb] * w[0] + ax[3 * bb + 1] * w[1] + ax[3 * bb + 2] * w[2]) / l;
    if (cb >= ca[bb]) return true;
    double sb = std::sqrt(std::max(0.0, 1 - cb * cb));
    double cosd = cb * ca[bb] + sb * sa[bb], sind = sb * ca[bb] - cb * sa[bb];
    return cosd >= 0 && sind <= R / l;
  };
  double lo3[3] = {1e300, 1e300, 1e300}, hi3[3] = {-1e300, -1e300, -1e300};
  for (int k : b.leaf_idx) {
    const double c[3] = {sph[k].cx, sph[k].cy, sph[k].cz};
    for (int q = 0; q < 3; ++q) {
      lo3[q] = std::min(lo3[q], c[q] - std::fabs(sph[k].r) - b.pad);
      hi3[q] = std::max(hi3[q], c[q] + std::fabs(sph[k].r) + b.pad);
    }
  }
  long dim3[3];
  for (int q = 0; q < 3; ++q) lo3[q] -= g, hi3[q] += g;  // one cell of margin: origins on surfaces around
  for (int q = 0; q < 3; ++q) dim3[q] = (long)std::ceil((hi3[q] - lo3[q]) / g);
  if (cellmode) printf("cells %ld x %ld x %ld\n", dim3[0], dim3[1], dim3[2]);
  std::map<std::pair<long, int>, std::vector<int>> memo;  // (patch id, bin) -> list (-1: overflow)
  auto list_for = [&](long pid, int bb, const double apex[3], double widen, int self) {
    auto key = std::make_pair(pid, bb);
    auto it = memo.find(key);
    if (it != memo.end()) return it->second;
    std::vector<int> L;
    if (self >= 0) L.push_back(self);
    for (int k : b.leaf_idx) {
      if (k == self) continue;
      if (meets(bb, apex, sph[k], std::fabs(sph[k].r) + 1.5 * b.pad + widen)) {
        L.push_back(k);
        if ((int)L.size() > kMax) break;
      }
    }
    if ((int)L.size() > kMax) L.assign(1, -1);
    memo[key] = L;
    return L;
  };
  FILE* f = fopen(path, "rb");
  if (!f) return 1;
  double w[9], prev[9] = {0};
  long walked = 0, wg = 0, ws = 0, res_g = 0, res_s = 0, bad = 0;
  double box_all = 0, box_g = 0, box_s = 0, tests_g = 0, tests_s = 0, box_res = 0;
  std::vector<long> hist_g(kMax + 2), hist_s(kMax + 2);
  while (fread(w, sizeof w, 1, f) == 1) {
    const bool bounce = w[8] >= 1;
    const int from = bounce ? (int)prev[7] : -2;
    for (int q = 0; q < 9; ++q) prev[q] = w[q];
    if (!bounce) continue;
    const double o[3] = {w[0], w[1], w[2]}, d[3] = {w[3], w[4], w[5]};
    double bt = INFINITY, t;
    int bi = -1;
    for (int q : b.big_idx)
      if (sph_hit(sph[q], o, d, 0.001, bt, t)) bt = t, bi = q;
    if (bt < INFINITY) continue;
    ++walked;
    long c1 = 0;
    double bt1 = bt;
    int bi1 = bi;
    for (int node = walk0; node < m;) {
      const psrt::BvhNode& nd = b.nodes[node];
      ++c1;
      if (!box(nd, o, d, bt1)) {
        node = nd.skip;
        continue;
      }
      if (nd.leaf >= 0) {
        for (int e = (nd.leaf >> 8); e < (nd.leaf >> 8) + (nd.leaf & 255); ++e) {
          int k = b.leaf_idx[e];
          if (sph_hit(sph[k], o, d, 0.001, bt1, t) && (t < bt1 || k > bi1)) bt1 = t, bi1 = k;
        }
        node = nd.skip;
      } else {
        node = node + 1;
      }
    }
    box_all += c1;
    const int bb = bin_of(d);
    std::vector<int> L;
    if (cellmode) {
      // 3-D cells of edge g over the BVH spheres' bounds, for every origin
      long ci[3];
      bool inside = true;
      for (int q = 0; q < 3; ++q) {
        ci[q] = (long)std::floor((o[q] - lo3[q]) / g);
        inside = inside && ci[q] >= 0 && ci[q] < dim3[q];
      }
      auto& hist = from == ground ? hist_g : hist_s;
      if (from == ground) ++wg, box_g += c1;
      else ++ws, box_s += c1;
      if (!inside) { hist[kMax + 1]++; continue; }
      const double apex[3] = {lo3[0] + (ci[0] + 0.5) * g, lo3[1] + (ci[1] + 0.5) * g, lo3[2] + (ci[2] + 0.5) * g};
      L = list_for((ci[0] * dim3[1] + ci[1]) * dim3[2] + ci[2], bb, apex, g * 0.8661 + 1e-3, -1);
    } else if (from == ground) {
      ++wg;
      box_g += c1;
      const long cx = (long)std::floor(o[0] / g), cz = (long)std::floor(o[2] / g);
      // apex: the patch centre on the ground surface; widen by the half-diagonal
      double apex[3] = {(cx + 0.5) * g, 0.0, (cz + 0.5) * g};
      const rt_sphere& G = sph[ground];
      double hx = apex[0] - G.cx, hz = apex[2] - G.cz;
      apex[1] = G.cy + std::sqrt(std::max(0.0, G.r * G.r - hx * hx - hz * hz));
      L = list_for((cx + 100000) * 1000000 + (cz + 100000), bb, apex, g * 0.7072 + 1e-3, -1);
    } else if (from >= 0) {
      ++ws;
      box_s += c1;
      const double apex[3] = {sph[from].cx, sph[from].cy, sph[from].cz};
      L = list_for(-1 - from, bb, apex, std::fabs(sph[from].r), from);
    } else {
      continue;
    }
    const bool ok = L.empty() || L[0] >= 0;
    auto& hist = from == ground ? hist_g : hist_s;
    hist[ok ? L.size() : kMax + 1]++;
    if (!ok) continue;
    if (bi1 >= 0 && std::find(L.begin(), L.end(), bi1) == L.end()) ++bad;
    if (from == ground) ++res_g, tests_g += L.size();
    else ++res_s, tests_s += L.size();
    box_res += c1;
  }
  printf("N=%d g=%.2f: walked %ld (box tests %.1f / ray); from the ground %ld, from BVH spheres %ld\n", N, g,
         walked, box_all / walked, wg, ws);
  printf("  ground: lists <= %d resolve %ld = %.1f%% (mean list %.2f); BVH: %ld = %.1f%% (mean %.2f); "
         "resolved %.1f%% of walked rays; unlisted true hits %ld\n", kMax, res_g, 100.0 * res_g / std::max(1L, wg),
         tests_g / std::max(1L, res_g), res_s, 100.0 * res_s / std::max(1L, ws), tests_s / std::max(1L, res_s),
         100.0 * (res_g + res_s) / walked, bad);
  printf("  box tests per walked ray: ground %.1f, BVH %.1f; resolved rays hold %.1f%% of the walk's box tests\n",
         box_g / std::max(1L, wg), box_s / std::max(1L, ws), 100.0 * box_res / box_all);
  printf("  list-size histogram ground:");
  for (int k = 0; k <= kMax + 1; ++k) printf(" %ld", hist_g[k]);
  printf("  (last: overflow)\n  list-size histogram BVH:   ");
  for (int k = 0; k <= kMax + 1; ++k) printf(" %ld", hist_s[k]);
  printf("\n  table entries built %zu\n", memo.size());
  return 0;
}
