// psrt/render.hpp — drop-in replacement for the reference pixel loop
// (programs/main.cc:70-88) over the C ABI of include/rt.h.
//
//   hittable_list world;                        // built with the usual API
//   world.add(make_shared<sphere>(point3(0,0,-1), 0.5));
//   camera cam;
//   psrt::frame f = psrt::render(world, cam, 400, 225, 100, 50);
//   psrt::write_ppm(std::cout, f);               // P3, exactly main.cc:70 + write_color
//
// psrt::flatten walks world.objects (hittable_list.h:40) in order, recursing
// into nested hittable_lists (a nested list's closest-hit scan is the same
// scan continued, so flattening keeps hittable_list::hit's result) and
// packing every sphere's (centre, radius) — any other hittable is an error.
#pragma once

#include <algorithm>
#include <memory>
#include <new>
#include <cstdint>
#include <ostream>
#include <stdexcept>
#include <string>
#include <vector>

#include "../rt.h"
#include "rtweekend.hpp"

namespace psrt {

// Page-locked host memory (rt_host_alloc, include/rt.h) as a std allocator:
// a frame held in it is written by the device directly, with no copy
// (DESIGN.md §7 "Host buffers"). Pinning is slow: keep such a frame and
// render into it again (render_into).
template <class T>
struct pinned_allocator {
  using value_type = T;
  pinned_allocator() = default;
  template <class U>
  pinned_allocator(const pinned_allocator<U>&) noexcept {}
  T* allocate(size_t n) {
    void* p = nullptr;
    if (rt_host_alloc(n * sizeof(T), &p) != RT_OK || (!p && n)) throw std::bad_alloc();
    return static_cast<T*>(p);
  }
  void deallocate(T* p, size_t) noexcept { rt_host_free(p); }
  template <class U>
  bool operator==(const pinned_allocator<U>&) const noexcept { return true; }
  template <class U>
  bool operator!=(const pinned_allocator<U>&) const noexcept { return false; }
};

template <template <class> class Alloc>
struct basic_frame {
  int width = 0, height = 0, rows = 0, spp = 0;
  std::vector<double, Alloc<double>> accum;        // rows x width x 3, reference order (top row first)
  std::vector<unsigned char, Alloc<unsigned char>> rgb8;  // write_color bytes
  rt_stats stats{};
  // false: render_into (one device) fetches the bytes alone, what main.cc
  // prints; the FP64 sums stay on the device (C3: 2.9 MB over the link, not 26)
  bool want_accum = true;
  // sizes the buffers for a shard (no reallocation when they already fit)
  void shape(int w, int h, int samples, int row_offset, int row_stride) {
    width = w, height = h, spp = samples;
    rows = std::max(0, rt_rows_owned(h, row_offset, row_stride));  // a shard may own none
    accum.resize(want_accum ? (size_t)rows * w * 3 : 0);
    rgb8.resize((size_t)rows * w * 3);
  }
};
using frame = basic_frame<std::allocator>;          // ordinary (pageable) memory
using pinned_frame = basic_frame<pinned_allocator>;  // page-locked: no device-to-host copy

inline void flatten_into(const hittable_list& list, std::vector<rt_sphere>& out) {
  for (const auto& obj : list.objects) {
    if (const auto* s = dynamic_cast<const sphere*>(obj.get())) {
      out.push_back(rt_sphere{s->centre.x(), s->centre.y(), s->centre.z(), s->radius});
    } else if (const auto* l = dynamic_cast<const hittable_list*>(obj.get())) {
      flatten_into(*l, out);
    } else {
      throw std::invalid_argument("psrt::flatten: only sphere and hittable_list are supported");
    }
  }
}

inline std::vector<rt_sphere> flatten(const hittable_list& world) {
  std::vector<rt_sphere> out;
  flatten_into(world, out);
  return out;
}

inline rt_camera to_rt(const camera& cam) {
  rt_camera c{};
  for (int k = 0; k < 3; ++k) {
    c.origin[k] = cam.origin[k];
    c.lower_left[k] = cam.lower_left_corner[k];
    c.horizontal[k] = cam.horizontal[k];
    c.vertical[k] = cam.vertical[k];
  }
  return c;
}

inline void check(int rc, const char* what) {
  if (rc != RT_OK) throw std::runtime_error(std::string(what) + ": " + rt_last_error());
}

// The structs of this header (rt_stats grew in ABI 5) must be the loaded
// library's: a libpsrt.so of another RT_ABI_VERSION is refused before any
// call could write past a caller's struct.
inline void check_abi() {
  static const int v = rt_abi_version();
  if (v != RT_ABI_VERSION)
    throw std::runtime_error("libpsrt.so ABI version " + std::to_string(v) + ", header " +
                             std::to_string(RT_ABI_VERSION));
}

// main.cc:72-88 for output rows row_offset, row_offset+row_stride, ...,
// into f (a pinned_frame kept across frames takes the frame with no copy)
template <class F>
inline void render_into(F& f, const hittable_list& world, const camera& cam, int width, int height,
                        int spp, int max_depth, uint64_t seed = 0, int row_offset = 0,
                        int row_stride = 1) {
  check_abi();
  const std::vector<rt_sphere> spheres = flatten(world);
  const rt_camera c = to_rt(cam);
  rt_params p{};
  p.width = width;
  p.height = height;
  p.spp = spp;
  p.max_depth = max_depth;
  p.seed = seed;
  p.row_offset = row_offset;
  p.row_stride = row_stride;
  f.shape(width, height, spp, row_offset, row_stride);
  check(rt_render(spheres.data(), (int)spheres.size(), &c, &p,
                  f.want_accum ? f.accum.data() : nullptr, f.rgb8.data(), &f.stats),
        "rt_render");
}

inline frame render(const hittable_list& world, const camera& cam, int width, int height,
                    int spp, int max_depth, uint64_t seed = 0, int row_offset = 0,
                    int row_stride = 1) {
  frame f;
  render_into(f, world, cam, width, height, spp, max_depth, seed, row_offset, row_stride);
  return f;
}

// ---- several devices (rt_group, include/rt.h) --------------
// One context and one host thread per member; interleaved rows gathered into
// reference pixel order in host memory; the same bits for any member count.
//
//   psrt::device_group g({0, 1, 2, 3, 4, 5, 6, 7});   // one member per GPU
//   g.set_scene(world, cam);
//   psrt::frame f = g.render(3840, 2160, 500, 50);    // repeat with new seeds
class device_group {
 public:
  explicit device_group(const std::vector<int>& devices) {
    check_abi();
    check(rt_group_create(devices.data(), (int)devices.size(), &g_), "rt_group_create");
  }
  ~device_group() { rt_group_destroy(g_); }
  device_group(const device_group&) = delete;
  device_group& operator=(const device_group&) = delete;
  int size() const { return rt_group_size(g_); }
  rt_context* context(int member) { return rt_group_context(g_, member); }
  void set_scene(const std::vector<rt_sphere>& spheres, const rt_camera& cam) {
    check(rt_group_set_scene(g_, spheres.data(), (int)spheres.size(), &cam), "rt_group_set_scene");
  }
  void set_scene(const hittable_list& world, const camera& cam) {
    set_scene(flatten(world), to_rt(cam));
  }
  template <class F>
  void render_into(F& f, int width, int height, int spp, int max_depth, uint64_t seed = 0,
                   int row_offset = 0, int row_stride = 1, unsigned flags = 0) {
    rt_params p{};
    p.width = width;
    p.height = height;
    p.spp = spp;
    p.max_depth = max_depth;
    p.seed = seed;
    p.row_offset = row_offset;
    p.row_stride = row_stride;
    p.flags = flags;
    f.want_accum = true;  // a group gathers the sums too
    f.shape(width, height, spp, row_offset, row_stride);
    check(rt_group_render(g_, &p, f.accum.data(), f.rgb8.data(), &f.stats), "rt_group_render");
  }
  frame render(int width, int height, int spp, int max_depth, uint64_t seed = 0,
               int row_offset = 0, int row_stride = 1, unsigned flags = 0) {
    frame f;
    render_into(f, width, height, spp, max_depth, seed, row_offset, row_stride, flags);
    return f;
  }

 private:
  rt_group* g_ = nullptr;
};

// main.cc:72-88 over several devices (one-shot: the group lives for one frame)
inline frame render(const hittable_list& world, const camera& cam, int width, int height,
                    int spp, int max_depth, const std::vector<int>& devices, uint64_t seed = 0,
                    int row_offset = 0, int row_stride = 1) {
  device_group g(devices);
  g.set_scene(world, cam);
  return g.render(width, height, spp, max_depth, seed, row_offset, row_stride);
}

// The book's material integrator and thin lens (extension):
// rt_render_materials over flattened spheres, one rt_material each.
inline frame render_materials(const std::vector<rt_sphere>& spheres,
                              const std::vector<rt_material>& mats, const rt_camera_lens& cam,
                              int width, int height, int spp, int max_depth, uint64_t seed = 0,
                              int row_offset = 0, int row_stride = 1) {
  check_abi();
  if (mats.size() != spheres.size())
    throw std::runtime_error("render_materials: one material per sphere");
  rt_params p{};
  p.width = width;
  p.height = height;
  p.spp = spp;
  p.max_depth = max_depth;
  p.seed = seed;
  p.row_offset = row_offset;
  p.row_stride = row_stride;
  p.flags = RT_FLAG_MATERIALS;
  frame f;
  f.shape(width, height, spp, row_offset, row_stride);
  check(rt_render_materials(spheres.data(), mats.data(), (int)spheres.size(), &cam, &p,
                            f.accum.data(), f.rgb8.data(), &f.stats),
        "rt_render_materials");
  return f;
}

// ---- scene files (rt_scene_load; DESIGN.md §Scene files) --------------------
struct scene_file {
  std::vector<rt_sphere> spheres;  // hittable_list order
  rt_camera cam{};
  rt_params params{};  // width/height/spp/max_depth/seed as the file states
};

inline scene_file load_scene(const std::string& path, const rt_params& defaults = rt_params{}) {
  scene_file s;
  s.params = defaults;
  rt_params scratch = defaults;
  const int n = rt_scene_load(path.c_str(), nullptr, 0, &s.cam, &scratch);
  if (n < 0) check(n, "rt_scene_load");
  s.spheres.resize(n);
  check(rt_scene_load(path.c_str(), s.spheres.data(), n, &s.cam, &s.params) < 0
            ? RT_E_SCENE : RT_OK,
        "rt_scene_load");
  return s;
}

inline std::string format_scene(const std::vector<rt_sphere>& spheres, const rt_camera& cam,
                                const rt_params* params = nullptr) {
  const long long len =
      rt_scene_format(spheres.data(), (int)spheres.size(), &cam, params, nullptr, 0);
  if (len < 0) check((int)len, "rt_scene_format");
  std::string text((size_t)len + 1, '\0');
  rt_scene_format(spheres.data(), (int)spheres.size(), &cam, params, &text[0], text.size());
  text.resize((size_t)len);
  return text;
}

// The reference-API world and camera for a loaded scene (hittable_list of
// spheres in file order; camera with the file's basis).
inline hittable_list to_world(const std::vector<rt_sphere>& spheres) {
  hittable_list world;
  for (const rt_sphere& q : spheres)
    world.add(make_shared<sphere>(point3(q.cx, q.cy, q.cz), q.r));
  return world;
}

inline camera to_camera(const rt_camera& c) {
  camera cam;
  cam.origin = point3(c.origin[0], c.origin[1], c.origin[2]);
  cam.lower_left_corner = point3(c.lower_left[0], c.lower_left[1], c.lower_left[2]);
  cam.horizontal = vec3(c.horizontal[0], c.horizontal[1], c.horizontal[2]);
  cam.vertical = vec3(c.vertical[0], c.vertical[1], c.vertical[2]);
  cam.aspect_ratio = cam.horizontal.length() / cam.vertical.length();
  return cam;
}

// "P3\n<w> <rows>\n255\n" then one "r g b" line per pixel (main.cc:70, color.h:21-23)
template <class F>
inline void write_ppm(std::ostream& out, const F& f) {
  out << "P3\n" << f.width << ' ' << f.rows << "\n255\n";
  for (size_t k = 0; k < f.rgb8.size(); k += 3)
    out << (int)f.rgb8[k] << ' ' << (int)f.rgb8[k + 1] << ' ' << (int)f.rgb8[k + 2] << '\n';
}

// P6 (binary) variant of the same image
template <class F>
inline void write_ppm_binary(std::ostream& out, const F& f) {
  out << "P6\n" << f.width << ' ' << f.rows << "\n255\n";
  out.write(reinterpret_cast<const char*>(f.rgb8.data()), (std::streamsize)f.rgb8.size());
}

}  // namespace psrt
