// psrt_scene.cpp — host-side scene and camera helpers of the C ABI
// (include/rt.h): the reference's camera() and two-sphere world, the look-at
// camera and final random-spheres scene the north star asks for (absent from
// the reference), and the host write_color epilogue.
#include <cmath>
#include <cstdint>
#include <cstring>

#include "../../include/rt.h"

namespace {

struct d3 {
  double x, y, z;
};
inline d3 operator+(d3 a, d3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline d3 operator-(d3 a, d3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline d3 operator*(double t, d3 a) { return {t * a.x, t * a.y, t * a.z}; }
inline d3 over(d3 a, double t) { return (1 / t) * a; }  // vec3.h:151-154
inline double len(d3 a) { return std::sqrt(a.x * a.x + a.y * a.y + a.z * a.z); }
inline d3 unit(d3 a) { return over(a, len(a)); }  // vec3.h:172-175
inline d3 cross(d3 u, d3 v) {
  return {u.y * v.z - u.z * v.y, u.z * v.x - u.x * v.z, u.x * v.y - u.y * v.x};
}

void put(rt_camera* c, d3 org, d3 llc, d3 h, d3 v) {
  const d3* src[4] = {&org, &llc, &h, &v};
  double* dst[4] = {c->origin, c->lower_left, c->horizontal, c->vertical};
  for (int k = 0; k < 4; ++k) {
    dst[k][0] = src[k]->x;
    dst[k][1] = src[k]->y;
    dst[k][2] = src[k]->z;
  }
}

// glibc rand() after srand(seed): the TYPE_3 additive lagged-Fibonacci
// generator r[i] = r[i-3] + r[i-31] (mod 2^32), output r >> 1, with the
// first 310 outputs discarded. The final scene is defined on this stream.
class GlibcStream {
 public:
  explicit GlibcStream(unsigned seed) {
    if (seed == 0) seed = 1;
    int32_t w = (int32_t)seed;
    r_[0] = w;
    for (int i = 1; i < 31; ++i) {
      int64_t t = (16807LL * (int64_t)r_[i - 1]) % 2147483647LL;
      if (t < 0) t += 2147483647LL;
      r_[i] = (int32_t)t;
    }
    pos_ = 0;
    for (int i = 0; i < 310; ++i) next();
  }
  int32_t next() {
    // ring of 31 words: word (pos+3) absorbs word pos (separation 3)
    const int a = (int)((pos_ + 3) % 31), b = (int)(pos_ % 31);
    const uint32_t v = (uint32_t)r_[a] + (uint32_t)r_[b];
    r_[a] = (int32_t)v;
    ++pos_;
    return (int32_t)(v >> 1);
  }
  double uniform() { return (double)next() / 2147483648.0; }

 private:
  int32_t r_[31];
  long pos_;
};

}  // namespace

extern "C" {

int rt_camera_default(rt_camera* out) {
  if (!out) return RT_E_INVALID;
  // camera.h:11-23
  const double aspect = 16.0 / 9.0;
  const double vh = 2.0, vw = vh * aspect, focal = 1.0;
  const d3 org{0, 0, 0}, h{vw, 0, 0}, v{0, vh, 0};
  const d3 llc = ((org - over(h, 2.0)) - over(v, 2.0)) + d3{0, 0, -focal};
  put(out, org, llc, h, v);
  return RT_OK;
}

int rt_camera_look_at(const double lookfrom[3], const double lookat[3], const double vup[3],
                      double vfov_deg, double aspect, rt_camera* out) {
  if (!lookfrom || !lookat || !vup || !out || !(aspect > 0)) return RT_E_INVALID;
  const double theta = vfov_deg * 3.1415926535897932385 / 180.0;  // raytracer.h:15-17
  const double vh = 2.0 * std::tan(theta / 2);
  const double vw = aspect * vh;
  const d3 from{lookfrom[0], lookfrom[1], lookfrom[2]};
  const d3 at{lookat[0], lookat[1], lookat[2]};
  const d3 up{vup[0], vup[1], vup[2]};
  const d3 w = unit(from - at);
  const d3 u = unit(cross(up, w));
  const d3 v = cross(w, u);
  const d3 h = vw * u, vv = vh * v;
  const d3 llc = ((from - over(h, 2.0)) - over(vv, 2.0)) - w;
  put(out, from, llc, h, vv);
  return RT_OK;
}

// The book's thin-lens camera (Ray Tracing in One Weekend v3.2, ch. 12), in
// the reference's vec3 arithmetic: horizontal = (focus_dist * vw) * u, etc.
int rt_camera_look_at_lens(const double lookfrom[3], const double lookat[3], const double vup[3],
                           double vfov_deg, double aspect, double aperture, double focus_dist,
                           rt_camera_lens* out) {
  if (!lookfrom || !lookat || !vup || !out || !(aspect > 0) || !(aperture >= 0) ||
      !(focus_dist > 0))
    return RT_E_INVALID;
  const double theta = vfov_deg * 3.1415926535897932385 / 180.0;  // raytracer.h:15-17
  const double vh = 2.0 * std::tan(theta / 2);
  const double vw = aspect * vh;
  const d3 from{lookfrom[0], lookfrom[1], lookfrom[2]};
  const d3 at{lookat[0], lookat[1], lookat[2]};
  const d3 up{vup[0], vup[1], vup[2]};
  const d3 w = unit(from - at);
  const d3 u = unit(cross(up, w));
  const d3 v = cross(w, u);
  const d3 h = (focus_dist * vw) * u, vv = (focus_dist * vh) * v;
  const d3 llc = ((from - over(h, 2.0)) - over(vv, 2.0)) - focus_dist * w;
  put(&out->base, from, llc, h, vv);
  out->u[0] = u.x, out->u[1] = u.y, out->u[2] = u.z;
  out->v[0] = v.x, out->v[1] = v.y, out->v[2] = v.z;
  out->lens_radius = aperture / 2;
  return RT_OK;
}

// The book's random_scene() (ch. 13) with materials, on the glibc srand(seed)
// stream. Every vec3 built from draws takes them in g++'s order (constructor
// arguments right to left: z, then y, then x), and color::random() *
// color::random() evaluates its right operand first.
int rt_scene_book_final(unsigned int seed, rt_sphere* out, rt_material* mats, int cap) {
  GlibcStream g(seed);
  int n = 0;
  auto push = [&](double x, double y, double z, double r, rt_material m) {
    if (out && n < cap) out[n] = rt_sphere{x, y, z, r};
    if (mats && n < cap) mats[n] = m;
    ++n;
  };
  auto lam = [](double r, double gg, double b) {
    return rt_material{RT_MAT_LAMBERTIAN, 0, {r, gg, b}, 0.0, 0.0};
  };
  auto rnd3 = [&](double lo, double hi, double c[3]) {  // vec3::random(lo, hi): z, y, x
    c[2] = lo + (hi - lo) * g.uniform();
    c[1] = lo + (hi - lo) * g.uniform();
    c[0] = lo + (hi - lo) * g.uniform();
  };
  push(0.0, -1000.0, 0.0, 1000.0, lam(0.5, 0.5, 0.5));
  for (int a = -11; a < 11; ++a) {
    for (int b = -11; b < 11; ++b) {
      const double choose = g.uniform();
      const double cz = b + 0.9 * g.uniform();  // point3(a + 0.9 rd, 0.2, b + 0.9 rd): z first
      const double cx = a + 0.9 * g.uniform();
      const d3 c{cx, 0.2, cz};
      if (!(len(c - d3{4, 0.2, 0}) > 0.9)) continue;
      if (choose < 0.8) {  // diffuse: albedo = color::random() * color::random()
        double rb[3], ra[3];
        rnd3(0.0, 1.0, rb);  // the right operand is evaluated first
        rnd3(0.0, 1.0, ra);
        push(cx, 0.2, cz, 0.2, lam(ra[0] * rb[0], ra[1] * rb[1], ra[2] * rb[2]));
      } else if (choose < 0.95) {  // metal
        double al[3];
        rnd3(0.5, 1.0, al);
        const double fuzz = 0.0 + (0.5 - 0.0) * g.uniform();
        push(cx, 0.2, cz, 0.2, rt_material{RT_MAT_METAL, 0, {al[0], al[1], al[2]}, fuzz, 0.0});
      } else {  // glass
        push(cx, 0.2, cz, 0.2, rt_material{RT_MAT_DIELECTRIC, 0, {1.0, 1.0, 1.0}, 0.0, 1.5});
      }
    }
  }
  push(0.0, 1.0, 0.0, 1.0, rt_material{RT_MAT_DIELECTRIC, 0, {1.0, 1.0, 1.0}, 0.0, 1.5});
  push(-4.0, 1.0, 0.0, 1.0, lam(0.4, 0.2, 0.1));
  push(4.0, 1.0, 0.0, 1.0, rt_material{RT_MAT_METAL, 0, {0.7, 0.6, 0.5}, 0.0, 0.0});
  return n;
}

int rt_scene_two_spheres(rt_sphere* out, int cap) {
  // main.cc:62-63
  const rt_sphere s[2] = {{0.0, 0.0, -1.0, 0.5}, {0.0, -100.5, 0.0, 100.0}};
  if (out)
    for (int k = 0; k < 2 && k < cap; ++k) out[k] = s[k];
  return 2;
}

int rt_scene_random_spheres(unsigned int seed, rt_sphere* out, int cap) {
  GlibcStream g(seed);
  int n = 0;
  auto push = [&](double x, double y, double z, double r) {
    if (out && n < cap) out[n] = rt_sphere{x, y, z, r};
    ++n;
  };
  push(0.0, -1000.0, 0.0, 1000.0);
  for (int a = -11; a < 11; ++a) {
    for (int b = -11; b < 11; ++b) {
      (void)g.uniform();  // choose_mat (diffuse-only scene: drawn, unused)
      const double cx = a + 0.9 * g.uniform();
      const double cz = b + 0.9 * g.uniform();
      const d3 c{cx, 0.2, cz};
      if (len(c - d3{4, 0.2, 0}) > 0.9) push(cx, 0.2, cz, 0.2);
    }
  }
  push(0.0, 1.0, 0.0, 1.0);
  push(-4.0, 1.0, 0.0, 1.0);
  push(4.0, 1.0, 0.0, 1.0);
  return n;
}

// color.h:8-24 on host accumulators (epilogue for gathered frames).
int rt_quantize_ppm(const double* accum, int width, int rows, int spp, unsigned char* rgb8) {
  if (!accum || !rgb8 || width <= 0 || rows < 0 || spp <= 0) return RT_E_INVALID;
  const double inv = 1.0 / spp;
  const size_t n = (size_t)width * rows * 3;
  for (size_t k = 0; k < n; ++k) {
    double x = std::sqrt(accum[k] * inv);
    x = (x < 0.0) ? 0.0 : x;
    x = (0.999 < x) ? 0.999 : x;
    rgb8[k] = (unsigned char)(int)(255.999 * x);
  }
  return RT_OK;
}

}  // extern "C"
