// Reads KAT lines ("n  cx cy cz r ...  ox oy oz dx dy dz  tmin tmax", hex floats)
// and prints hittable_list::hit through the host API of include/psrt/rtweekend.hpp
// ("index px py pz nx ny nz t front_face"), plus nested-list flattening checks.
#include <cstdio>
#include <fstream>
#include <iostream>
#include <sstream>
#include <string>

#include "psrt/render.hpp"

int main(int argc, char** argv) {
  std::ifstream in(argv[1]);
  std::string line;
  while (std::getline(in, line)) {
    if (line.empty()) continue;
    std::istringstream ss(line);
    auto rd = [&]() { std::string t; ss >> t; return std::strtod(t.c_str(), nullptr); };
    int n = (int)rd();
    hittable_list world;
    std::vector<shared_ptr<sphere>> sp;
    for (int k = 0; k < n; ++k) {
      double cx = rd(), cy = rd(), cz = rd(), r = rd();
      sp.push_back(make_shared<sphere>(point3(cx, cy, cz), r));
      world.add(sp.back());
    }
    double ox = rd(), oy = rd(), oz = rd(), dx = rd(), dy = rd(), dz = rd();
    double tmin = rd(), tmax = rd();
    ray r(point3(ox, oy, oz), vec3(dx, dy, dz));
    hit_record rec;
    if (!world.hit(r, tmin, tmax, rec)) { std::printf("-1\n"); continue; }
    int idx = -1;
    double closest = tmax;
    hit_record tmp;
    for (int k = 0; k < n; ++k)
      if (sp[k]->hit(r, tmin, closest, tmp)) { closest = tmp.t; idx = k; }
    std::printf("%d %a %a %a %a %a %a %a %d\n", idx, rec.p.x(), rec.p.y(), rec.p.z(),
                rec.normal.x(), rec.normal.y(), rec.normal.z(), rec.t, (int)rec.front_face);
  }
  // flatten: nested lists keep order; a non-sphere hittable is rejected
  hittable_list inner;
  inner.add(make_shared<sphere>(point3(1, 2, 3), 4));
  inner.add(make_shared<sphere>(point3(5, 6, 7), 8));
  hittable_list outer;
  outer.add(make_shared<sphere>(point3(0, 0, 0), 1));
  outer.add(make_shared<hittable_list>(inner));
  outer.add(make_shared<sphere>(point3(9, 9, 9), 2));
  auto flat = psrt::flatten(outer);
  std::printf("flat %zu", flat.size());
  for (auto& s : flat) std::printf(" %g,%g,%g,%g", s.cx, s.cy, s.cz, s.r);
  std::printf("\n");
  struct other : hittable {
    bool hit(const ray&, double, double, hit_record&) const override { return false; }
  };
  hittable_list bad;
  bad.add(make_shared<other>());
  try { psrt::flatten(bad); std::printf("bad accepted\n"); }
  catch (const std::invalid_argument&) { std::printf("bad rejected\n"); }
  return 0;
}
