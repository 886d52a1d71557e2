// ORACLE — test infrastructure only. Builds the reference's own hot path
// (programs/main.cc ray_color, sphere.cc, hittable_list.cc, vec3.h, camera.h,
// color.h, random.h — compiled unmodified from /root/reference by
// oracle/Makefile into oracle/_ref/ref_render) behind a parameterised driver.
//
// What the driver adds around the reference code:
//  * `#define main reference_main` so the reference main() stays callable
//    (--reference-main runs it verbatim: 400x225, 100 spp, P3 to stdout).
//  * rand() interposition: the reference calls glibc rand() through
//    random_double() (random.h:4-14). In --rng glibc mode rand() is glibc's
//    own generator (random(), which glibc's rand() wraps); in --rng counter
//    mode it returns the per-(pixel, sample) counter stream (xorshift32 + Weyl) of
//    oracle/oracle_rng.h, reseeded before each sample — the device contract.
//  * A copy of the main.cc:72-88 pixel loop with W/H/spp/depth/shard
//    parameters, calling the reference ray_color() and write_color().
//  * The final random-spheres scene and look-at camera (not in the
//    reference), built with the reference vec3/sphere/
//    hittable_list/random_double.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <chrono>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#define main reference_main
#include "main.cc"
#undef main

#include "oracle_rng.h"

static int g_counter_mode = 0;
static uint64_t g_counter_state = 0;

extern "C" int rand(void) noexcept {
  if (g_counter_mode) return oracle_counter_rand(&g_counter_state);
  return (int)random();  // glibc: rand() is (int) __random ()
}

namespace {

struct counting_world : public hittable {
  const hittable& inner;
  mutable uint64_t calls = 0;
  explicit counting_world(const hittable& w) : inner(w) {}
  bool hit(const ray& r, double tmin, double tmax, hit_record& rec) const override {
    ++calls;
    return inner.hit(r, tmin, tmax, rec);
  }
};

// Known-answer mode: each input line is "n  cx cy cz r (n times)  ox oy oz
// dx dy dz  tmin tmax" (hex floats); each output line is the reference
// hittable_list::hit result "index px py pz nx ny nz t front_face" (hex
// floats; index -1 = miss). The hit sphere's index is recovered by running
// sphere::hit per object with the final t (the reference records no index).
int run_kat(const std::string& path) {
  std::ifstream in(path);
  std::string line;
  while (std::getline(in, line)) {
    if (line.empty()) continue;
    std::istringstream ss(line);
    auto rd = [&]() { std::string t; ss >> t; return std::strtod(t.c_str(), nullptr); };
    int n = (int)rd();
    hittable_list world;
    std::vector<std::shared_ptr<sphere>> sp;
    for (int k = 0; k < n; ++k) {
      double cx = rd(), cy = rd(), cz = rd(), r = rd();
      sp.push_back(make_shared<sphere>(point3(cx, cy, cz), r));
      world.add(sp.back());
    }
    double ox = rd(), oy = rd(), oz = rd(), dx = rd(), dy = rd(), dz = rd();
    double tmin = rd(), tmax = rd();
    ray r(point3(ox, oy, oz), vec3(dx, dy, dz));
    hit_record rec;
    if (!world.hit(r, tmin, tmax, rec)) {
      std::printf("-1\n");
      continue;
    }
    // which object produced rec: replay the list scan (hittable_list.cc:9-17)
    int idx = -1;
    double closest = tmax;
    hit_record tmp;
    for (int k = 0; k < n; ++k)
      if (sp[k]->hit(r, tmin, closest, tmp)) { closest = tmp.t; idx = k; }
    std::printf("%d %a %a %a %a %a %a %a %d\n", idx, rec.p.x(), rec.p.y(), rec.p.z(),
                rec.normal.x(), rec.normal.y(), rec.normal.z(), rec.t, (int)rec.front_face);
  }
  return 0;
}

// Known-answer mode over one scene: the first line of the file is
// "n  cx cy cz r (n times)", every further line one ray "ox oy oz dx dy dz
// tmin tmax" (hex floats); output as run_kat, one line per ray. For ray sets
// too large to repeat the sphere list on every line (tests/golden/
// make_culling_kat.py: tens of thousands of rays on the 485-sphere scene).
int run_kat_scene(const std::string& path) {
  std::ifstream in(path);
  std::string line;
  if (!std::getline(in, line)) return 2;
  std::istringstream hs(line);
  auto rdh = [&]() { std::string t; hs >> t; return std::strtod(t.c_str(), nullptr); };
  const int n = (int)rdh();
  hittable_list world;
  std::vector<std::shared_ptr<sphere>> sp;
  for (int k = 0; k < n; ++k) {
    double cx = rdh(), cy = rdh(), cz = rdh(), r = rdh();
    sp.push_back(make_shared<sphere>(point3(cx, cy, cz), r));
    world.add(sp.back());
  }
  while (std::getline(in, line)) {
    if (line.empty()) continue;
    std::istringstream ss(line);
    auto rd = [&]() { std::string t; ss >> t; return std::strtod(t.c_str(), nullptr); };
    double ox = rd(), oy = rd(), oz = rd(), dx = rd(), dy = rd(), dz = rd();
    double tmin = rd(), tmax = rd();
    ray r(point3(ox, oy, oz), vec3(dx, dy, dz));
    hit_record rec;
    if (!world.hit(r, tmin, tmax, rec)) {
      std::printf("-1\n");
      continue;
    }
    int idx = -1;  // which object produced rec: replay the list scan (hittable_list.cc:9-17)
    double closest = tmax;
    hit_record tmp;
    for (int k = 0; k < n; ++k)
      if (sp[k]->hit(r, tmin, closest, tmp)) { closest = tmp.t; idx = k; }
    std::printf("%d %a %a %a %a %a %a %a %d\n", idx, rec.p.x(), rec.p.y(), rec.p.z(),
                rec.normal.x(), rec.normal.y(), rec.normal.z(), rec.t, (int)rec.front_face);
  }
  return 0;
}

void usage() {
  std::fprintf(stderr,
               "ref_render [--reference-main] [--width W] [--height H] [--spp S]\n"
               "  [--depth D] [--scene two|final] [--scene-seed N] [--rng glibc|counter]\n"
               "  [--seed N] [--rows OFF:STRIDE[:COUNT]] [--accum FILE] [--ppm FILE]\n"
               "  [--dump-scene FILE] [--camera default|lookat] [--kat FILE] [--kat-scene FILE]\n"
               "  [--cols C0:C1]\n");
}

}  // namespace

int main(int argc, char** argv) {
  int W = 400, H = -1, spp = 10, depth = 50, row_off = 0, row_stride = 1, row_count = -1;
  int col0 = 0, col1 = -1;  // --cols: render only columns [col0, col1) of each row
  unsigned scene_seed = 1;
  uint64_t seed = 0;
  std::string scene = "two", rng = "counter", accum_path, ppm_path, dump_path, cam_kind, kat_path,
      kat_scene_path;
  bool run_reference_main = false;
  for (int a = 1; a < argc; ++a) {
    std::string k = argv[a];
    auto next = [&]() -> std::string {
      if (a + 1 >= argc) { usage(); std::exit(2); }
      return argv[++a];
    };
    if (k == "--reference-main") run_reference_main = true;
    else if (k == "--width") W = std::stoi(next());
    else if (k == "--height") H = std::stoi(next());
    else if (k == "--spp") spp = std::stoi(next());
    else if (k == "--depth") depth = std::stoi(next());
    else if (k == "--scene") scene = next();
    else if (k == "--scene-seed") scene_seed = (unsigned)std::stoul(next());
    else if (k == "--rng") rng = next();
    else if (k == "--seed") seed = std::stoull(next());
    else if (k == "--accum") accum_path = next();
    else if (k == "--ppm") ppm_path = next();
    else if (k == "--dump-scene") dump_path = next();
    else if (k == "--camera") cam_kind = next();
    else if (k == "--kat") kat_path = next();
    else if (k == "--kat-scene") kat_scene_path = next();
    else if (k == "--cols") {
      std::string v = next();
      if (std::sscanf(v.c_str(), "%d:%d", &col0, &col1) != 2) { usage(); return 2; }
    }
    else if (k == "--rows") {
      std::string v = next();
      if (std::sscanf(v.c_str(), "%d:%d:%d", &row_off, &row_stride, &row_count) < 2) { usage(); return 2; }
    } else { usage(); return 2; }
  }
  if (run_reference_main) return reference_main();
  if (!kat_path.empty()) return run_kat(kat_path);
  if (!kat_scene_path.empty()) return run_kat_scene(kat_scene_path);

  // ---- world (main.cc:61-63, or the final scene) ----
  hittable_list world;
  std::vector<std::shared_ptr<sphere>> spheres;
  if (scene == "two") {
    spheres.push_back(make_shared<sphere>(point3(0, 0, -1), 0.5));
    spheres.push_back(make_shared<sphere>(point3(0, -100.5, 0), 100.0));
  } else if (scene == "final") {
    srandom(scene_seed);
    g_counter_mode = 0;
    spheres.push_back(make_shared<sphere>(point3(0, -1000, 0), 1000));
    for (int a = -11; a < 11; a++) {
      for (int b = -11; b < 11; b++) {
        auto choose = random_double();
        (void)choose;
        double cx = a + 0.9 * random_double();
        double cz = b + 0.9 * random_double();
        point3 centre(cx, 0.2, cz);
        if ((centre - point3(4, 0.2, 0)).length() > 0.9)
          spheres.push_back(make_shared<sphere>(centre, 0.2));
      }
    }
    spheres.push_back(make_shared<sphere>(point3(0, 1, 0), 1.0));
    spheres.push_back(make_shared<sphere>(point3(-4, 1, 0), 1.0));
    spheres.push_back(make_shared<sphere>(point3(4, 1, 0), 1.0));
  } else { usage(); return 2; }
  for (auto& s : spheres) world.add(s);

  // ---- camera ----
  camera cam;  // camera.h:11-23
  if (cam_kind.empty()) cam_kind = (scene == "final") ? "lookat" : "default";
  if (H < 0) H = (cam_kind == "default") ? (int)(W / cam.aspect_ratio) : (int)(W / 1.5);
  if (cam_kind == "lookat") {
    // book camera(lookfrom (13,2,3), lookat 0, vup (0,1,0), vfov 20, W/H), no defocus
    point3 lookfrom(13, 2, 3), lookat(0, 0, 0);
    vec3 vup(0, 1, 0);
    double aspect = (double)W / H;
    auto theta = degrees_to_radians(20.0);
    auto hh = tan(theta / 2);
    auto vh = 2.0 * hh;
    auto vw = aspect * vh;
    auto w = unit_vector(lookfrom - lookat);
    auto u = unit_vector(cross(vup, w));
    auto v = cross(w, u);
    cam.aspect_ratio = aspect;
    cam.origin = lookfrom;
    cam.horizontal = vw * u;
    cam.vertical = vh * v;
    cam.lower_left_corner = cam.origin - cam.horizontal / 2 - cam.vertical / 2 - w;
  }

  if (!dump_path.empty()) {
    FILE* f = std::fopen(dump_path.c_str(), "w");
    std::fprintf(f, "spheres %zu\n", spheres.size());
    for (auto& s : spheres)
      std::fprintf(f, "%a %a %a %a\n", s->centre.x(), s->centre.y(), s->centre.z(), s->radius);
    std::fprintf(f, "camera\n%a %a %a\n%a %a %a\n%a %a %a\n%a %a %a\n", cam.origin.x(),
                 cam.origin.y(), cam.origin.z(), cam.lower_left_corner.x(),
                 cam.lower_left_corner.y(), cam.lower_left_corner.z(), cam.horizontal.x(),
                 cam.horizontal.y(), cam.horizontal.z(), cam.vertical.x(), cam.vertical.y(),
                 cam.vertical.z());
    std::fclose(f);
  }

  // ---- pixel loop (main.cc:70-88) ----
  const bool counter = (rng == "counter");
  if (!counter && (row_off != 0 || row_stride != 1 || row_count >= 0)) {
    std::fprintf(stderr, "glibc stream needs the whole frame\n");
    return 2;
  }
  if (!counter) { srandom(1); g_counter_mode = 0; } else g_counter_mode = 1;
  int rows = (H - 1 - row_off) / row_stride + 1;
  if (row_count >= 0 && row_count < rows) rows = row_count;
  counting_world counted(world);
  if (col1 < 0 || col1 > W) col1 = W;
  if (col0 < 0) col0 = 0;
  const int ncols = col1 > col0 ? col1 - col0 : 0;
  std::vector<double> accum((size_t)rows * ncols * 3);
  std::ostringstream ppm;
  ppm << "P3\n" << ncols << ' ' << rows << "\n255\n";
  auto t0 = std::chrono::steady_clock::now();
  for (int k = 0; k < rows; ++k) {
    int j = H - 1 - (row_off + k * row_stride);
    for (int i = col0; i < col1; ++i) {
      color pixel_color(0, 0, 0);
      for (int s = 0; s < spp; ++s) {
        if (counter) g_counter_state = oracle_stream_state(seed, (uint32_t)(j * W + i), (uint32_t)s);
        double u = ((double)i + random_double()) / (W - 1);
        double v = ((double)j + random_double()) / (H - 1);
        pixel_color += ray_color(cam.get_ray(u, v), counted, depth);
      }
      double* px = &accum[((size_t)k * ncols + (i - col0)) * 3];
      px[0] = pixel_color.x(), px[1] = pixel_color.y(), px[2] = pixel_color.z();
      write_color(ppm, pixel_color, spp);
    }
  }
  double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  std::fprintf(stderr, "{\"samples\": %llu, \"rays\": %llu, \"seconds\": %.6f}\n",
               (unsigned long long)rows * ncols * spp, (unsigned long long)counted.calls, secs);
  if (!accum_path.empty()) {
    FILE* f = std::fopen(accum_path.c_str(), "wb");
    std::fwrite(accum.data(), sizeof(double), accum.size(), f);
    std::fclose(f);
  }
  if (!ppm_path.empty()) {
    std::ofstream(ppm_path) << ppm.str();
  } else if (accum_path.empty() && dump_path.empty()) {
    std::cout << ppm.str();
  }
  return 0;
}
