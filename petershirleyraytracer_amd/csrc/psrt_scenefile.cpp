// psrt_scenefile.cpp — scene/camera fixture files: a
// line-oriented text form of what main.cc:53-63 builds in code (the world's
// spheres in hittable_list order, the camera, and the pixel-loop parameters).
//
//   psrt-scene 1
//   # comment (to end of line)
//   camera default                                   # camera.h:11-23
//   camera basis  ox oy oz  lx ly lz  hx hy hz  vx vy vz
//   camera look_at fx fy fz  ax ay az  ux uy uz  vfov_deg  aspect|auto
//   render width W height H spp S depth D seed X     # any subset, any order
//   sphere cx cy cz r                                # one per object, in order
//
// Numbers are C99 decimal or hexadecimal floating literals (strtod), so a file
// written by rt_scene_format (%.17g) reads back bit-identical. `aspect auto`
// is width / height of the render parameters. Sphere order is kept: it is
// hittable_list::hit's tie-break (hittable_list.cc:9-17).
#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/rt.h"
#include "psrt_error.h"

namespace {

struct Parser {
  const char* p;
  int line = 1;

  void skip_blank() {
    while (*p == ' ' || *p == '\t' || *p == '\r') ++p;
    if (*p == '#')
      while (*p && *p != '\n') ++p;
  }
  bool at_eol() {
    skip_blank();
    return *p == '\n' || *p == '\0';
  }
  void next_line() {
    while (*p && *p != '\n') ++p;
    if (*p == '\n') ++p, ++line;
  }
  // the next whitespace-delimited word on this line ("" at end of line)
  std::string word() {
    skip_blank();
    const char* b = p;
    while (*p && *p != ' ' && *p != '\t' && *p != '\r' && *p != '\n' && *p != '#') ++p;
    return std::string(b, p);
  }
  bool number(double& out) {
    const std::string w = word();
    if (w.empty()) return false;
    char* end = nullptr;
    errno = 0;
    out = std::strtod(w.c_str(), &end);
    return end == w.c_str() + w.size();
  }
  bool integer(long long& out) {
    const std::string w = word();
    if (w.empty()) return false;
    char* end = nullptr;
    errno = 0;
    out = std::strtoll(w.c_str(), &end, 0);
    return errno == 0 && end == w.c_str() + w.size();
  }
  bool uinteger(unsigned long long& out) {
    const std::string w = word();
    if (w.empty() || w[0] == '-') return false;
    char* end = nullptr;
    errno = 0;
    out = std::strtoull(w.c_str(), &end, 0);
    return errno == 0 && end == w.c_str() + w.size();
  }
};

int bad(int line, const char* what) {
  return psrt::set_error(RT_E_SCENE, "scene file line %d: %s", line, what);
}

void put_vec(std::string& s, const char* sep, const double* v) {
  char buf[96];
  std::snprintf(buf, sizeof buf, "%s%.17g %.17g %.17g", sep, v[0], v[1], v[2]);
  s += buf;
}

}  // namespace

extern "C" {

int rt_scene_parse(const char* text, rt_sphere* out, int cap, rt_camera* cam, rt_params* params) {
  if (!text || cap < 0 || (cap > 0 && !out))
    return psrt::set_error(RT_E_INVALID, "rt_scene_parse: bad arguments");
  Parser ps{text};
  bool header = false, have_cam = false, look_at = false, auto_aspect = false;
  double la[11] = {0};  // lookfrom, lookat, vup, vfov, aspect
  rt_camera c{};
  long long width = -1, height = -1, spp = -1, depth = -2;
  unsigned long long seed = 0;
  bool have_seed = false;
  long long n = 0;
  for (; *ps.p; ps.next_line()) {
    if (ps.at_eol()) continue;
    const std::string kw = ps.word();
    if (!header) {
      long long ver = 0;
      if (kw != "psrt-scene" || !ps.integer(ver) || ver != 1 || !ps.at_eol())
        return bad(ps.line, "expected header 'psrt-scene 1'");
      header = true;
      continue;
    }
    if (kw == "sphere") {
      double v[4];
      for (double& x : v)
        if (!ps.number(x)) return bad(ps.line, "sphere needs cx cy cz r");
      if (!ps.at_eol()) return bad(ps.line, "trailing text after sphere");
      if (n >= (1LL << 30)) return bad(ps.line, "too many spheres");
      if (n < cap) out[n] = rt_sphere{v[0], v[1], v[2], v[3]};
      ++n;
    } else if (kw == "camera") {
      if (have_cam) return bad(ps.line, "second camera line");
      have_cam = true;
      const std::string kind = ps.word();
      if (kind == "default") {
        rt_camera_default(&c);
      } else if (kind == "basis") {
        double* dst[4] = {c.origin, c.lower_left, c.horizontal, c.vertical};
        for (double* d : dst)
          for (int k = 0; k < 3; ++k)
            if (!ps.number(d[k])) return bad(ps.line, "camera basis needs 12 numbers");
      } else if (kind == "look_at") {
        look_at = true;
        for (int k = 0; k < 10; ++k)
          if (!ps.number(la[k]))
            return bad(ps.line, "camera look_at needs lookfrom lookat vup vfov aspect");
        const char* save = ps.p;
        if (ps.word() == "auto") {
          auto_aspect = true;
        } else {
          ps.p = save;
          if (!ps.number(la[10]) || !(la[10] > 0))
            return bad(ps.line, "camera look_at aspect must be > 0 or 'auto'");
        }
      } else {
        return bad(ps.line, "camera must be default, basis or look_at");
      }
      if (!ps.at_eol()) return bad(ps.line, "trailing text after camera");
    } else if (kw == "render") {
      while (!ps.at_eol()) {
        const std::string key = ps.word();
        long long v = 0;
        if (key == "seed") {
          if (!ps.uinteger(seed)) return bad(ps.line, "render seed needs an unsigned integer");
          have_seed = true;
          continue;
        }
        if (!ps.integer(v)) return bad(ps.line, "render keys take integer values");
        if (key == "width" && v > 0 && v <= (1 << 20)) width = v;
        else if (key == "height" && v > 0 && v <= (1 << 20)) height = v;
        else if (key == "spp" && v > 0 && v <= (1LL << 30)) spp = v;
        else if (key == "depth" && v >= -1 && v <= 100000) depth = v;
        else return bad(ps.line, "render key unknown or value out of range");
      }
    } else {
      return bad(ps.line, "unknown keyword (expected sphere, camera or render)");
    }
  }
  if (!header) return bad(ps.line, "empty scene file (no 'psrt-scene 1' header)");

  rt_params pl = params ? *params : rt_params{};
  if (width > 0) pl.width = (int)width;
  if (height > 0) pl.height = (int)height;
  if (spp > 0) pl.spp = (int)spp;
  if (depth >= -1) pl.max_depth = (int)depth;
  if (have_seed) pl.seed = seed;
  if (!have_cam) rt_camera_default(&c);
  if (look_at) {
    if (auto_aspect) {
      if (pl.width <= 0 || pl.height <= 0)
        return psrt::set_error(RT_E_SCENE, "scene file: 'aspect auto' needs width and height");
      la[10] = (double)pl.width / pl.height;
    }
    bool finite = rt_camera_look_at(la, la + 3, la + 6, la[9], la[10], &c) == RT_OK;
    const double* basis[4] = {c.origin, c.lower_left, c.horizontal, c.vertical};
    for (const double* b : basis)
      for (int k = 0; k < 3; ++k) finite = finite && std::isfinite(b[k]);
    if (!finite) return psrt::set_error(RT_E_SCENE, "scene file: degenerate look_at camera");
  }
  if (params) *params = pl;
  if (cam) *cam = c;
  return (int)n;
}

int rt_scene_load(const char* path, rt_sphere* out, int cap, rt_camera* cam, rt_params* params) {
  if (!path) return psrt::set_error(RT_E_INVALID, "rt_scene_load: null path");
  FILE* f = std::fopen(path, "rb");
  if (!f) return psrt::set_error(RT_E_INVALID, "rt_scene_load: cannot open %s", path);
  std::string text;
  char buf[1 << 16];
  size_t got;
  while ((got = std::fread(buf, 1, sizeof buf, f)) > 0) text.append(buf, got);
  const bool err = std::ferror(f) != 0;
  std::fclose(f);
  if (err) return psrt::set_error(RT_E_INVALID, "rt_scene_load: read error on %s", path);
  if (text.find('\0') != std::string::npos)
    return psrt::set_error(RT_E_SCENE, "rt_scene_load: %s is not a text scene file", path);
  return rt_scene_parse(text.c_str(), out, cap, cam, params);
}

long long rt_scene_format(const rt_sphere* spheres, int n, const rt_camera* cam,
                          const rt_params* params, char* buf, size_t cap) {
  if (n < 0 || (n > 0 && !spheres))
    return psrt::set_error(RT_E_INVALID, "rt_scene_format: bad sphere list");
  std::string s = "psrt-scene 1\n";
  char line[160];
  std::snprintf(line, sizeof line, "# %d spheres\n", n);
  s += line;
  if (cam) {
    s += "camera basis";
    put_vec(s, " ", cam->origin);
    put_vec(s, "  ", cam->lower_left);
    put_vec(s, "  ", cam->horizontal);
    put_vec(s, "  ", cam->vertical);
    s += "\n";
  }
  if (params) {
    std::snprintf(line, sizeof line, "render width %d height %d spp %d depth %d seed %llu\n",
                  params->width, params->height, params->spp, params->max_depth,
                  (unsigned long long)params->seed);
    s += line;
  }
  for (int k = 0; k < n; ++k) {
    const rt_sphere& q = spheres[k];
    std::snprintf(line, sizeof line, "sphere %.17g %.17g %.17g %.17g\n", q.cx, q.cy, q.cz, q.r);
    s += line;
  }
  if (buf && cap > 0) {
    const size_t m = s.size() < cap - 1 ? s.size() : cap - 1;
    std::memcpy(buf, s.data(), m);
    buf[m] = '\0';
  }
  return (long long)s.size();
}

}  // extern "C"
