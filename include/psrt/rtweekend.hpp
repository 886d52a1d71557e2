// psrt/rtweekend.hpp — the reference's host-side C++ API surface, in one header.
//
// Same class/function names, signatures and IEEE operation order as the
// reference headers (programs/vec3.h, ray.h, hittable.h, sphere.h/.cc,
// hittable_list.h/.cc, camera.h, color.h, random.h, raytracer.h), so code
// written against the reference compiles against this. The per-name headers
// in include/raytracer/ forward here. The render hot path does NOT run through
// these host classes: psrt/render.hpp flattens a hittable_list into the C ABI
// (include/rt.h) and the gfx950 megakernel traces it.
//
// Differences from the reference, all deliberate:
//   * random_double() uses the intended scaling rand()/(RAND_MAX + 1.0)
//     (random.h:7 overflows int and never terminates).
//   * vec3::random(min,max) draws z, then y, then x explicitly — the order
//     g++ gives the reference's unspecified argument evaluation (vec3.h:78-81).
//   * write_color is inline (color.h:8 defines a non-inline function in a
//     header: an ODR violation when included twice).
//   * camera gains a look-at constructor (the final scene's camera; no defocus).
#pragma once

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <iostream>
#include <limits>
#include <memory>
#include <vector>

using std::make_shared;
using std::shared_ptr;
using std::sqrt;

// ---- raytracer.h: constants and utilities ----------------------------------
const double infinity = std::numeric_limits<double>::infinity();
const double pi = 3.1415926535897932385;

inline double degrees_to_radians(double degrees) { return degrees * pi / 180.0; }

template <class T>
inline T clamp(const T v, const T lo, const T hi) {
  return std::min(std::max(v, lo), hi);
}

// ---- random.h --------------------------------------------------------------
inline double random_double() { return (double)rand() / (RAND_MAX + 1.0); }

inline double random_double(double min, double max) {
  return min + (max - min) * random_double();
}

// ---- vec3.h -----------------------------------------------------------------
class vec3 {
 public:
  double e[3];

  vec3() : e{0, 0, 0} {}
  vec3(double e0, double e1, double e2) : e{e0, e1, e2} {}

  double x() const { return e[0]; }
  double y() const { return e[1]; }
  double z() const { return e[2]; }

  vec3 operator-() const { return vec3(-e[0], -e[1], -e[2]); }
  double operator[](int i) const { return e[i]; }
  double& operator[](int i) { return e[i]; }

  vec3& operator+=(const vec3& o) {
    for (int k = 0; k < 3; ++k) e[k] += o.e[k];
    return *this;
  }
  vec3& operator*=(const double t) {
    for (int k = 0; k < 3; ++k) e[k] *= t;
    return *this;
  }
  vec3& operator/=(const double t) { return *this *= 1 / t; }

  double length_squared() const { return e[0] * e[0] + e[1] * e[1] + e[2] * e[2]; }
  double length() const { return sqrt(length_squared()); }

  static vec3 random() {
    const double z = random_double(), y = random_double(), x = random_double();
    return vec3(x, y, z);
  }
  static vec3 random(double min, double max) {
    const double z = random_double(min, max);
    const double y = random_double(min, max);
    const double x = random_double(min, max);
    return vec3(x, y, z);
  }
  // rejection sampling in the cube [-1,1)^3, accepting length_squared <= 1
  static vec3 random_in_unit_sphere();
  static vec3 random_unit_vector();
  static vec3 random_in_hemisphere(const vec3& normal);
};

using point3 = vec3;
using color = vec3;

inline std::ostream& operator<<(std::ostream& out, const vec3& v) {
  return out << v[0] << ' ' << v[1] << ' ' << v[2];
}
inline vec3 operator+(const vec3& a, const vec3& b) {
  return vec3(a[0] + b[0], a[1] + b[1], a[2] + b[2]);
}
inline vec3 operator-(const vec3& a, const vec3& b) {
  return vec3(a[0] - b[0], a[1] - b[1], a[2] - b[2]);
}
inline vec3 operator*(const double t, const vec3& v) { return vec3(t * v[0], t * v[1], t * v[2]); }
inline vec3 operator*(const vec3& a, const vec3& b) {
  return vec3(a[0] * b[0], a[1] * b[1], a[2] * b[2]);
}
inline vec3 operator*(const vec3& v, const double t) { return t * v; }
inline vec3 operator/(const vec3& v, const double t) { return (1 / t) * v; }
inline double dot(const vec3& a, const vec3& b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
inline vec3 cross(const vec3& a, const vec3& b) {
  return vec3(a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]);
}
inline vec3 unit_vector(const vec3& v) { return v / v.length(); }

inline vec3 vec3::random_in_unit_sphere() {
  for (;;) {
    const vec3 v = random(-1.0, 1.0);
    if (!(v.length_squared() > 1.0)) return v;
  }
}
inline vec3 vec3::random_unit_vector() { return unit_vector(random_in_unit_sphere()); }
inline vec3 vec3::random_in_hemisphere(const vec3& normal) {
  const vec3 v = random_in_unit_sphere();
  return dot(v, normal) > 0 ? v : -v;
}

// ---- ray.h --------------------------------------------------------------------
class ray {
 public:
  point3 orig;
  vec3 dir;

  ray() {}
  ray(const point3& o, const vec3& d) : orig(o), dir(d) {}
  point3 origin() const { return orig; }
  vec3 direction() const { return dir; }
  point3 at(double t) const { return orig + dir * t; }
};

// ---- hittable.h ---------------------------------------------------------------
struct hit_record {
  point3 p;
  vec3 normal;
  double t;
  bool front_face;

  inline void set_face_normal(const ray& r, const vec3& outward_normal) {
    front_face = dot(r.direction(), outward_normal) < 0;
    normal = front_face ? outward_normal : -outward_normal;
  }
};

class hittable {
 public:
  virtual ~hittable() = default;
  virtual bool hit(const ray& r, double tmin, double tmax, hit_record& record) const = 0;
};

// ---- sphere.h / sphere.cc -------------------------------------------------------
class sphere : public hittable {
 public:
  point3 centre;
  double radius;

  sphere() : centre(0, 0, 0), radius(0) {}
  sphere(const point3& c, double r) : centre(c.x(), c.y(), c.z()), radius(r) {}

  bool hit(const ray& r, double tmin, double tmax, hit_record& record) const override {
    const vec3 d = r.direction();
    const vec3 oc = r.origin() - centre;
    const double a = dot(d, d);
    const double half_b = dot(d, oc);
    const double c = dot(oc, oc) - radius * radius;
    const double disc = half_b * half_b - a * c;
    if (disc < 0) return false;
    const double root = std::sqrt(disc);
    double t = (-half_b - root) / a;
    if (t < tmin || t > tmax) {
      t = (-half_b + root) / a;
      if (t < tmin || t > tmax) return false;
    }
    record.p = r.at(t);
    record.set_face_normal(r, (record.p - centre) / radius);
    record.t = t;
    return true;
  }
};

// ---- hittable_list.h / .cc -------------------------------------------------------
class hittable_list : public hittable {
 public:
  std::vector<shared_ptr<hittable>> objects;

  hittable_list() {}
  hittable_list(shared_ptr<hittable> object) { add(object); }
  virtual ~hittable_list() { clear(); }

  void add(shared_ptr<hittable> object) { objects.push_back(object); }
  void clear() { objects.clear(); }

  bool hit(const ray& r, double tmin, double tmax, hit_record& record) const override {
    hit_record probe;
    bool any = false;
    double closest = tmax;
    for (const auto& obj : objects) {
      if (!obj->hit(r, tmin, closest, probe)) continue;
      any = true;
      closest = probe.t;
      record = probe;
    }
    return any;
  }
};

// ---- camera.h ---------------------------------------------------------------------
class camera {
 public:
  double aspect_ratio;
  point3 origin;
  vec3 horizontal;
  vec3 vertical;
  vec3 lower_left_corner;

  // the reference's fixed 16:9 pinhole at the origin looking down -z
  camera() {
    aspect_ratio = 16.0 / 9.0;
    const double vh = 2.0;
    const double vw = vh * aspect_ratio;
    const double focal = 1.0;
    origin = point3(0, 0, 0);
    horizontal = vec3(vw, 0, 0);
    vertical = vec3(0, vh, 0);
    lower_left_corner = origin - horizontal / 2.0 - vertical / 2.0 + vec3(0, 0, -focal);
  }

  // extension: look-at pinhole (vertical field of view in degrees), no defocus
  camera(point3 lookfrom, point3 lookat, vec3 vup, double vfov, double aspect) {
    aspect_ratio = aspect;
    const double vh = 2.0 * std::tan(degrees_to_radians(vfov) / 2);
    const double vw = aspect * vh;
    const vec3 w = unit_vector(lookfrom - lookat);
    const vec3 u = unit_vector(cross(vup, w));
    const vec3 v = cross(w, u);
    origin = lookfrom;
    horizontal = vw * u;
    vertical = vh * v;
    lower_left_corner = origin - horizontal / 2 - vertical / 2 - w;
  }

  ray get_ray(double u, double v) const {
    return ray(origin, lower_left_corner + horizontal * u + vertical * v - origin);
  }
};

// ---- color.h ------------------------------------------------------------------------
inline void write_color(std::ostream& out, const color& pixel_color, int samples_per_pixel) {
  const double scale = 1.0 / samples_per_pixel;
  for (int k = 0; k < 3; ++k) {
    const double g = sqrt(pixel_color[k] * scale);  // gamma 2
    out << (int)(255.999 * clamp(g, 0.0, 0.999)) << (k < 2 ? ' ' : '\n');
  }
}
