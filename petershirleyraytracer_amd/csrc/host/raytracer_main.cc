// raytracer — the reference's main() (programs/main.cc:51-92) on the MI355X
// hot path. The scene and camera are built with the reference API
// (include/raytracer/*.h); the pixel loop (main.cc:72-88) is replaced by
// psrt::render -> rt_render (include/rt.h) -> the gfx950 megakernel.
//
//   raytracer                       # main.cc as written: 400 wide, 16:9, 100 spp, depth 50
//   raytracer --scene final --width 1200 --height 800 --spp 100 -o out.ppm
//   raytracer --rows 1:8 ...        # one interleaved shard (rows 1, 9, 17, ...)
//   raytracer --devices 8 ...       # one frame over GPUs 0..7 (rt_group: a host
//                                   # thread and context per device, interleaved
//                                   # rows); --devices 0,0,1 lists members
//                                   # explicitly (a device may repeat)
//   raytracer --scene-file s.scene  # world/camera/parameters from a scene file;
//                                   # flags given on the command line win
//   raytracer --scene final --save-scene final.scene   # write the scene, render nothing
//   raytracer --scene book --width 1200 --height 800 --spp 10 [--aperture 0.1 --focus 10]
//                                   # the book's materials + thin lens
#include <cctype>
#include <cerrno>
#include <chrono>
#include <cstdio>
#include <climits>
#include <cstdlib>
#include <fstream>
#include <iostream>
#include <string>
#include <vector>

#include "psrt/render.hpp"
#include "raytracer/camera.h"
#include "raytracer/color.h"
#include "raytracer/hittable_list.h"
#include "raytracer/sphere.h"

namespace {

// The final random-spheres world (diffuse-only), with the
// reference API: glibc srand(seed), per cell a choose draw then x, z jitter.
void random_spheres(hittable_list& world, unsigned seed) {
  srand(seed);
  world.add(make_shared<sphere>(point3(0, -1000, 0), 1000));
  for (int a = -11; a < 11; a++) {
    for (int b = -11; b < 11; b++) {
      (void)random_double();  // choose_mat
      const double cx = a + 0.9 * random_double();
      const double cz = b + 0.9 * random_double();
      const point3 centre(cx, 0.2, cz);
      if ((centre - point3(4, 0.2, 0)).length() > 0.9) world.add(make_shared<sphere>(centre, 0.2));
    }
  }
  world.add(make_shared<sphere>(point3(0, 1, 0), 1.0));
  world.add(make_shared<sphere>(point3(-4, 1, 0), 1.0));
  world.add(make_shared<sphere>(point3(4, 1, 0), 1.0));
}

int usage() {
  std::fprintf(stderr,
               "raytracer [--scene two|final|book | --scene-file FILE] [--width W] [--height H]\n"
               "          [--spp S] [--depth D] [--seed N] [--rows OFF:STRIDE] [-o FILE] [--p6]\n"
               "          [--accum FILE] [--save-scene FILE] [--aperture A] [--focus F]\n"
               "          [--devices N | --devices D0,D1,...]\n");
  return 2;
}

// a decimal integer / an unsigned 64-bit integer / a floating-point number,
// the whole string, in range
bool parse_int(const char* s, int& out) {
  char* end = nullptr;
  errno = 0;
  const long v = std::strtol(s, &end, 10);
  if (end == s || *end != '\0' || errno == ERANGE || v < INT_MIN || v > INT_MAX) return false;
  out = (int)v;
  return true;
}
bool parse_u64(const char* s, unsigned long long& out) {
  char* end = nullptr;
  // digits only: strtoull would skip leading blanks and accept a sign, and
  // wrap " -1" to 2^64 - 1
  if (!std::isdigit((unsigned char)*s)) return false;
  errno = 0;
  out = std::strtoull(s, &end, 10);
  return end != s && *end == '\0' && errno != ERANGE;
}
bool parse_double(const char* s, double& out) {
  char* end = nullptr;
  errno = 0;
  out = std::strtod(s, &end);
  return end != s && *end == '\0' && errno != ERANGE;
}

// a non-negative decimal integer, the whole string
bool parse_index(const std::string& s, int& out) {
  if (s.empty() || s.size() > 6 || s.find_first_not_of("0123456789") != std::string::npos)
    return false;
  out = std::atoi(s.c_str());
  return true;
}

// --devices N (devices 0..N-1) | D0,D1,... (a member per entry; repeats allowed)
bool parse_devices(const std::string& v, std::vector<int>& out) {
  out.clear();
  if (v.find(',') == std::string::npos) {
    int n = 0;
    if (!parse_index(v, n) || n < 1 || n > 1024) return false;
    for (int d = 0; d < n; ++d) out.push_back(d);
    return true;
  }
  size_t a = 0;
  while (a <= v.size()) {
    const size_t b = std::min(v.find(',', a), v.size());
    int d = 0;
    if (!parse_index(v.substr(a, b - a), d)) return false;
    out.push_back(d);
    a = b + 1;
  }
  return !out.empty() && out.size() <= 1024;
}

}  // namespace

int main(int argc, char** argv) {
  std::string scene = "two", out_path, accum_path, scene_path, save_path;
  int width = 400, height = -1, spp = 100, depth = 50, row_off = 0, row_stride = 1;
  unsigned long long seed = 0;
  double aperture = 0.1, focus = 10.0;  // --scene book: the book's lens
  std::vector<int> devices;             // --devices: several members (rt_group)
  bool p6 = false, set_w = false, set_h = false, set_spp = false, set_depth = false,
       set_seed = false;
  for (int a = 1; a < argc; ++a) {
    const std::string k = argv[a];
    auto val = [&]() -> const char* { return a + 1 < argc ? argv[++a] : nullptr; };
    const char* v = nullptr;
    if (k == "--p6") { p6 = true; continue; }
    if (!(v = val())) return usage();
    if (k == "--scene") scene = v;
    else if (k == "--scene-file") scene_path = v;
    else if (k == "--save-scene") save_path = v;
    else if (k == "--width") { if (!parse_int(v, width)) return usage(); set_w = true; }
    else if (k == "--height") { if (!parse_int(v, height)) return usage(); set_h = true; }
    else if (k == "--spp") { if (!parse_int(v, spp)) return usage(); set_spp = true; }
    else if (k == "--depth") { if (!parse_int(v, depth)) return usage(); set_depth = true; }
    else if (k == "--seed") { if (!parse_u64(v, seed)) return usage(); set_seed = true; }
    else if (k == "-o") out_path = v;
    else if (k == "--accum") accum_path = v;
    else if (k == "--aperture") { if (!parse_double(v, aperture)) return usage(); }
    else if (k == "--focus") { if (!parse_double(v, focus)) return usage(); }
    else if (k == "--devices") {
      if (!parse_devices(v, devices)) return usage();
    }
    else if (k == "--rows") {
      const std::string r = v;
      const size_t c = r.find(':');
      if (c == std::string::npos || !parse_int(r.substr(0, c).c_str(), row_off) ||
          !parse_int(r.substr(c + 1).c_str(), row_stride))
        return usage();
    } else return usage();
  }

  // world + camera (main.cc:53-63)
  hittable_list world;
  camera cam;
  if (!scene_path.empty()) {
    try {
      rt_params defaults{};
      defaults.width = width;
      defaults.height = height;
      defaults.spp = spp;
      defaults.max_depth = depth;
      defaults.seed = seed;
      const psrt::scene_file sf = psrt::load_scene(scene_path, defaults);
      world = psrt::to_world(sf.spheres);
      cam = psrt::to_camera(sf.cam);
      if (!set_w) width = sf.params.width;
      if (!set_h) height = sf.params.height;
      if (!set_spp) spp = sf.params.spp;
      if (!set_depth) depth = sf.params.max_depth;
      if (!set_seed) seed = sf.params.seed;
      if (height < 0) height = (int)(width / cam.aspect_ratio);
    } catch (const std::exception& e) {
      std::cerr << "raytracer: " << e.what() << "\n";
      return 1;
    }
  } else if (scene == "two") {
    if (height < 0) height = (int)(width / cam.aspect_ratio);
    world.add(make_shared<sphere>(point3(0, 0, -1), 0.5));
    world.add(make_shared<sphere>(point3(0, -100.5, 0), 100.0));
  } else if (scene == "book") {
    if (height < 0) height = (int)(width / 1.5);
    if (!devices.empty()) {
      std::cerr << "raytracer: --devices renders the reference integrator only\n";
      return 2;
    }
  } else if (scene == "final") {
    if (height < 0) height = (int)(width / 1.5);
    random_spheres(world, 1);
    cam = camera(point3(13, 2, 3), point3(0, 0, 0), vec3(0, 1, 0), 20.0, (double)width / height);
  } else {
    return usage();
  }

  if (!save_path.empty()) {
    if (scene == "book") {
      std::cerr << "raytracer: scene files hold spheres only (no materials)\n";
      return 2;
    }
    try {
      rt_params p{};
      p.width = width;
      p.height = height;
      p.spp = spp;
      p.max_depth = depth;
      p.seed = seed;
      std::ofstream f(save_path, std::ios::binary);
      f << psrt::format_scene(psrt::flatten(world), psrt::to_rt(cam), &p);
      if (!f) throw std::runtime_error("cannot write " + save_path);
    } catch (const std::exception& e) {
      std::cerr << "raytracer: " << e.what() << "\n";
      return 1;
    }
    return 0;
  }

  try {
    const auto t0 = std::chrono::steady_clock::now();
    psrt::frame f;
    if (scene == "book" && scene_path.empty()) {
      // the book's random_scene() with materials, lookfrom (13,2,3), vfov 20
      const int n = rt_scene_book_final(1, nullptr, nullptr, 0);
      std::vector<rt_sphere> sph((size_t)n);
      std::vector<rt_material> mats((size_t)n);
      rt_scene_book_final(1, sph.data(), mats.data(), n);
      const double from[3] = {13, 2, 3}, at[3] = {0, 0, 0}, up[3] = {0, 1, 0};
      rt_camera_lens lc{};
      psrt::check(rt_camera_look_at_lens(from, at, up, 20.0, (double)width / height, aperture,
                                         focus, &lc),
                  "rt_camera_look_at_lens");
      f = psrt::render_materials(sph, mats, lc, width, height, spp, depth, seed, row_off,
                                 row_stride);
    } else if (!devices.empty()) {
      f = psrt::render(world, cam, width, height, spp, depth, devices, seed, row_off, row_stride);
    } else {
      // the bytes alone unless --accum asks for the sums (main.cc prints bytes)
      f.want_accum = !accum_path.empty();
      psrt::render_into(f, world, cam, width, height, spp, depth, seed, row_off, row_stride);
    }
    const double secs =
        std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    std::ofstream file;
    if (!out_path.empty()) file.open(out_path, std::ios::binary);
    std::ostream& out = out_path.empty() ? std::cout : file;
    if (p6)
      psrt::write_ppm_binary(out, f);
    else
      psrt::write_ppm(out, f);
    if (!accum_path.empty()) {
      std::ofstream acc(accum_path, std::ios::binary);
      acc.write(reinterpret_cast<const char*>(f.accum.data()),
                (std::streamsize)(f.accum.size() * sizeof(double)));
    }
    std::fprintf(stderr,
                 "{\"samples\": %llu, \"rays\": %llu, \"kernel_ms\": %.3f, \"wall_s\": %.4f, "
                 "\"msamples_per_s\": %.3f}\n",
                 (unsigned long long)f.stats.samples, (unsigned long long)f.stats.rays,
                 f.stats.kernel_ms, secs, f.stats.samples / secs / 1e6);
    std::cerr << "Done.\n";
  } catch (const std::exception& e) {
    std::cerr << "raytracer: " << e.what() << "\n";
    return 1;
  }
  return 0;
}
