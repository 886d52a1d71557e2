/*
 * ORACLE — test infrastructure only. Nothing in petershirleyraytracer_amd/
 * links, loads or calls this file; only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg use it, as the checker.
 *
 * A plain-C restatement of the reference hot path
 * (fengye/PeterShirleyRaytracer, /root/reference/programs), operation for
 * operation in IEEE binary64, built with -ffp-contract=off:
 *
 *   pixel loop ............ main.cc:72-88
 *   ray_color ............. main.cc:34-49   (recursion restated as a loop:
 *                           0.5*x is exact, so 0.5^k*sky == the recursion)
 *   hittable_list::hit .... hittable_list.cc:3-20
 *   sphere::hit ........... sphere.cc:3-40
 *   set_face_normal ....... hittable.h:14-18
 *   random_in_hemisphere .. vec3.h:102-109 -> random_in_unit_sphere vec3.h:83-95
 *                           -> vec3::random(min,max) vec3.h:78-81 (g++
 *                           evaluates the three constructor arguments right
 *                           to left: draw 1 -> z, 2 -> y, 3 -> x)
 *   random_double ......... random.h:4-14 (intended rand()/(RAND_MAX+1.0))
 *   camera::get_ray ....... camera.h:25-28, camera() camera.h:11-23
 *   unit_vector, dot, / ... vec3.h:151-175 (v/t is (1/t)*v)
 *   write_color ........... color.h:8-24
 *
 * Parity pins: tests/test_oracle.py checks this file against outputs of the
 * reference sources themselves (oracle/_ref/ref_render, built by
 * oracle/Makefile from /root/reference) and against tests/golden/ fixtures
 * generated from them (tests/golden/make_golden.py).
 */
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "../include/rt.h"
#include "oracle_rng.h"

#define ORACLE_RNG_COUNTER 0
#define ORACLE_RNG_GLIBC 1

typedef struct {
  double x, y, z;
} v3;

static inline v3 mk(double x, double y, double z) {
  v3 r;
  r.x = x;
  r.y = y;
  r.z = z;
  return r;
}
static inline v3 add(v3 a, v3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 sub(v3 a, v3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 scale(double t, v3 a) { return mk(t * a.x, t * a.y, t * a.z); }
static inline v3 neg(v3 a) { return mk(-a.x, -a.y, -a.z); }
static inline double dot3(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline v3 cross3(v3 u, v3 v) {
  return mk(u.y * v.z - u.z * v.y, u.z * v.x - u.x * v.z, u.x * v.y - u.y * v.x);
}
/* vec3.h:151-154: operator/(v, t) is (1/t) * v */
static inline v3 divs(v3 a, double t) { return scale(1.0 / t, a); }
/* vec3.h:63-71, 172-175 */
static inline v3 unit(v3 a) { return divs(a, sqrt(a.x * a.x + a.y * a.y + a.z * a.z)); }

/* ---- RNG -------------------------------------------------------------------- */
typedef struct {
  int mode;
  uint64_t counter_state;
  oracle_glibc_rand* glibc;
  uint64_t draws;
} orng;

static inline double random_double(orng* g) {
  int32_t v;
  g->draws++;
  if (g->mode == ORACLE_RNG_GLIBC)
    v = oracle_glibc_next(g->glibc);
  else
    v = oracle_counter_rand(&g->counter_state);
  return (double)v / (2147483647 + 1.0);
}

/* random.h:10-14 */
static inline double random_range(orng* g, double lo, double hi) {
  return lo + (hi - lo) * random_double(g);
}

/* vec3.h:78-81 with g++'s right-to-left argument evaluation */
static inline v3 random_vec(orng* g, double lo, double hi) {
  double z = random_range(g, lo, hi);
  double y = random_range(g, lo, hi);
  double x = random_range(g, lo, hi);
  return mk(x, y, z);
}

/* vec3.h:83-95 */
static inline v3 random_in_unit_sphere(orng* g) {
  for (;;) {
    v3 v = random_vec(g, -1.0, 1.0);
    if (v.x * v.x + v.y * v.y + v.z * v.z > 1.0) continue;
    return v;
  }
}

/* vec3.h:102-109 */
static inline v3 random_in_hemisphere(orng* g, v3 normal) {
  v3 v = random_in_unit_sphere(g);
  if (dot3(v, normal) > 0) return v;
  return neg(v);
}

/* ---- geometry ---------------------------------------------------------------- */
typedef struct {
  v3 p, normal;
  double t;
  int front_face;
  int index;
} hitrec;

/* sphere.cc:3-40 (+ hittable.h:14-18). Returns 1 on hit. */
static int sphere_hit(const rt_sphere* s, v3 o, v3 d, double tmin, double tmax,
                      hitrec* rec) {
  v3 c = mk(s->cx, s->cy, s->cz);
  v3 amc = sub(o, c);
  double A = dot3(d, d);
  double hb = dot3(d, amc);
  double C = dot3(amc, amc) - s->r * s->r;
  double disc = hb * hb - A * C;
  double sq, t;
  v3 outward;
  if (disc < 0) return 0;
  sq = sqrt(disc);
  t = (-hb - sq) / A;
  if (t < tmin || t > tmax) {
    t = (-hb + sq) / A;
    if (t < tmin || t > tmax) return 0;
  }
  rec->p = add(o, scale(t, d)); /* ray.h:25-28 at(t) = orig + dir*t */
  outward = divs(sub(rec->p, c), s->r);
  rec->front_face = dot3(d, outward) < 0;
  rec->normal = rec->front_face ? outward : neg(outward);
  rec->t = t;
  return 1;
}

/* hittable_list.cc:3-20 */
static int world_hit(const rt_sphere* sph, int n, v3 o, v3 d, double tmin,
                     double tmax, hitrec* rec) {
  hitrec tmp;
  int any = 0, k;
  double closest = tmax;
  for (k = 0; k < n; ++k) {
    if (sphere_hit(&sph[k], o, d, tmin, closest, &tmp)) {
      any = 1;
      closest = tmp.t;
      tmp.index = k;
      *rec = tmp;
    }
  }
  return any;
}

/* One bounce record for path-trace known-answer tests. */
typedef struct {
  double o[3], d[3];
  double t;
  int32_t index; /* -1 = miss */
  int32_t front_face;
  uint64_t draws_after; /* RNG draws consumed by the sample so far */
} oracle_bounce;

/* main.cc:34-49, iterative. Returns the sample colour in col; counts rays. */
static void ray_color(const rt_sphere* sph, int n, v3 o, v3 d, int max_depth,
                      orng* g, double col[3], uint64_t* rays,
                      oracle_bounce* trace, int trace_cap, int* trace_len) {
  int depth, k = 0;
  for (depth = max_depth;; --depth) {
    hitrec rec;
    int hit;
    if (depth < 0) { /* main.cc:36-37 */
      col[0] = col[1] = col[2] = 0.0;
      break;
    }
    ++*rays;
    hit = world_hit(sph, n, o, d, 0, INFINITY, &rec);
    if (trace && *trace_len < trace_cap) {
      oracle_bounce* b = &trace[*trace_len];
      b->o[0] = o.x, b->o[1] = o.y, b->o[2] = o.z;
      b->d[0] = d.x, b->d[1] = d.y, b->d[2] = d.z;
      b->t = hit ? rec.t : INFINITY;
      b->index = hit ? rec.index : -1;
      b->front_face = hit ? rec.front_face : 0;
    }
    if (hit) {
      /* main.cc:42-43: target = (p + normal) + random_in_hemisphere(normal) */
      v3 rv = random_in_hemisphere(g, rec.normal);
      v3 target = add(add(rec.p, rec.normal), rv);
      o = rec.p;
      d = sub(target, rec.p);
      ++k;
      if (trace && *trace_len < trace_cap) trace[*trace_len].draws_after = g->draws;
      if (trace) ++*trace_len;
      continue;
    }
    if (trace && *trace_len < trace_cap) trace[*trace_len].draws_after = g->draws;
    if (trace) ++*trace_len;
    {
      /* main.cc:46-48 */
      v3 ud = unit(d);
      double t = 0.5 * (ud.y + 1.0);
      v3 c = add(scale(1.0 - t, mk(1.0, 1.0, 1.0)), scale(t, mk(0.5, 0.7, 1.0)));
      int m;
      for (m = 0; m < k; ++m) c = scale(0.5, c); /* main.cc:43, unwound */
      col[0] = c.x, col[1] = c.y, col[2] = c.z;
    }
    break;
  }
}

/* camera.h:25-28 */
static inline void get_ray(const rt_camera* cam, double u, double v, v3* o, v3* d) {
  v3 org = mk(cam->origin[0], cam->origin[1], cam->origin[2]);
  v3 llc = mk(cam->lower_left[0], cam->lower_left[1], cam->lower_left[2]);
  v3 h = mk(cam->horizontal[0], cam->horizontal[1], cam->horizontal[2]);
  v3 vv = mk(cam->vertical[0], cam->vertical[1], cam->vertical[2]);
  *o = org;
  *d = sub(add(add(llc, scale(u, h)), scale(v, vv)), org);
}

/* main.cc:78-84 for one pixel */
static void render_pixel(const rt_sphere* sph, int n, const rt_camera* cam,
                         const rt_params* p, orng* g, int i, int j, double acc[3],
                         uint64_t* rays) {
  int s;
  acc[0] = acc[1] = acc[2] = 0.0;
  for (s = 0; s < p->spp; ++s) {
    double u, v, col[3];
    v3 o, d;
    if (g->mode == ORACLE_RNG_COUNTER)
      g->counter_state = oracle_stream_state(p->seed, (uint32_t)(j * p->width + i),
                                             (uint32_t)s);
    u = ((double)i + random_double(g)) / (p->width - 1);
    v = ((double)j + random_double(g)) / (p->height - 1);
    get_ray(cam, u, v, &o, &d);
    ray_color(sph, n, o, d, p->max_depth, g, col, rays, NULL, 0, NULL);
    acc[0] += col[0];
    acc[1] += col[1];
    acc[2] += col[2];
  }
}

/* color.h:8-24 */
static inline unsigned char quant(double c, int spp) {
  double x = sqrt(c * (1.0 / spp));
  if (x < 0.0) x = 0.0; /* clamp: std::min(std::max(v, lo), hi) */
  if (x > 0.999) x = 0.999;
  /* std::max(NaN, 0.0) returns NaN (first arg), std::min(NaN, .999) NaN */
  return (unsigned char)(int)(255.999 * x);
}

int oracle_quantize(const double* accum, int w, int rows, int spp, unsigned char* out) {
  size_t k, nn = (size_t)w * rows * 3;
  if (!accum || !out || w <= 0 || rows < 0 || spp <= 0) return RT_E_INVALID;
  for (k = 0; k < nn; ++k) out[k] = quant(accum[k], spp);
  return RT_OK;
}

typedef struct {
  const rt_sphere* sph;
  int n;
  const rt_camera* cam;
  const rt_params* p;
  double* accum;
  int rows_owned;
  int tid, nthreads;
  uint64_t rays;
} job;

static void* worker(void* arg) {
  job* jb = (job*)arg;
  orng g;
  int k, i;
  memset(&g, 0, sizeof g);
  g.mode = ORACLE_RNG_COUNTER;
  for (k = jb->tid; k < jb->rows_owned; k += jb->nthreads) {
    int r = jb->p->row_offset + k * jb->p->row_stride;
    int j = jb->p->height - 1 - r;
    for (i = 0; i < jb->p->width; ++i)
      render_pixel(jb->sph, jb->n, jb->cam, jb->p, &g, i, j,
                   &jb->accum[((size_t)k * jb->p->width + i) * 3], &jb->rays);
  }
  return NULL;
}

int oracle_rows_owned(int h, int off, int stride) {
  if (h <= 0 || stride <= 0 || off < 0 || off >= h) return 0;
  return (h - 1 - off) / stride + 1;
}

/* The pixel loop of main.cc:72-88 over the owned rows.
 * rng_mode GLIBC: one serial stream (seed = srand seed; reference default 1);
 * requires the full frame (row_offset 0, stride 1) and runs single-threaded.
 * rng_mode COUNTER: per-(pixel,sample) streams; `threads` workers over rows. */
int oracle_render(const rt_sphere* sph, int n, const rt_camera* cam,
                  const rt_params* p, int rng_mode, int threads, double* accum,
                  unsigned char* rgb8, uint64_t* rays_out) {
  int rows;
  if (!sph || n < 0 || !cam || !p || !accum) return RT_E_INVALID;
  if (p->width < 2 || p->height < 2 || p->spp <= 0 || p->max_depth < -1) return RT_E_INVALID;
  rows = oracle_rows_owned(p->height, p->row_offset, p->row_stride);
  if (rows <= 0) return RT_E_INVALID;
  if (rng_mode == ORACLE_RNG_GLIBC) {
    oracle_glibc_rand gl;
    orng g;
    uint64_t rays = 0;
    int k, i;
    if (p->row_offset != 0 || p->row_stride != 1) return RT_E_INVALID;
    oracle_glibc_srand(&gl, (unsigned)p->seed);
    memset(&g, 0, sizeof g);
    g.mode = ORACLE_RNG_GLIBC;
    g.glibc = &gl;
    for (k = 0; k < rows; ++k) {
      int j = p->height - 1 - k;
      for (i = 0; i < p->width; ++i)
        render_pixel(sph, n, cam, p, &g, i, j, &accum[((size_t)k * p->width + i) * 3], &rays);
    }
    if (rays_out) *rays_out = rays;
  } else {
    job jobs[256];
    pthread_t th[256];
    int t;
    uint64_t rays = 0;
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    for (t = 0; t < threads; ++t) {
      jobs[t].sph = sph, jobs[t].n = n, jobs[t].cam = cam, jobs[t].p = p;
      jobs[t].accum = accum, jobs[t].rows_owned = rows;
      jobs[t].tid = t, jobs[t].nthreads = threads, jobs[t].rays = 0;
    }
    if (threads == 1) {
      worker(&jobs[0]);
    } else {
      for (t = 0; t < threads; ++t) pthread_create(&th[t], NULL, worker, &jobs[t]);
      for (t = 0; t < threads; ++t) pthread_join(th[t], NULL);
    }
    for (t = 0; t < threads; ++t) rays += jobs[t].rays;
    if (rays_out) *rays_out = rays;
  }
  if (rgb8) oracle_quantize(accum, p->width, rows, p->spp, rgb8);
  return RT_OK;
}

/* Counter-mode samples of an explicit pixel list (for sampled parity at full
 * sizes): out[k*3..] = pixel_color of pixel (i[k], j[k]) over spp samples. */
int oracle_render_pixels(const rt_sphere* sph, int n, const rt_camera* cam,
                         const rt_params* p, const int* ii, const int* jj, int count,
                         double* out, uint64_t* rays_out) {
  orng g;
  uint64_t rays = 0;
  int k;
  if (!sph || !cam || !p || !ii || !jj || !out || count < 0) return RT_E_INVALID;
  memset(&g, 0, sizeof g);
  g.mode = ORACLE_RNG_COUNTER;
  for (k = 0; k < count; ++k)
    render_pixel(sph, n, cam, p, &g, ii[k], jj[k], &out[(size_t)k * 3], &rays);
  if (rays_out) *rays_out = rays;
  return RT_OK;
}

/* Path trace of one counter-mode sample (known-answer vectors). Returns the
 * number of bounce records (<= cap) and the sample colour in col. */
int oracle_trace_sample(const rt_sphere* sph, int n, const rt_camera* cam,
                        const rt_params* p, int i, int j, int s, double col[3],
                        oracle_bounce* trace, int cap) {
  orng g;
  uint64_t rays = 0;
  int len = 0;
  double u, v;
  v3 o, d;
  memset(&g, 0, sizeof g);
  g.mode = ORACLE_RNG_COUNTER;
  g.counter_state = oracle_stream_state(p->seed, (uint32_t)(j * p->width + i), (uint32_t)s);
  u = ((double)i + random_double(&g)) / (p->width - 1);
  v = ((double)j + random_double(&g)) / (p->height - 1);
  get_ray(cam, u, v, &o, &d);
  ray_color(sph, n, o, d, p->max_depth, &g, col, &rays, trace, cap, &len);
  return len;
}

/* sphere::hit known-answer: rec_out = {p[3], normal[3], t, front_face}. */
int oracle_sphere_hit(const rt_sphere* s, const double o[3], const double d[3],
                      double tmin, double tmax, double rec_out[8]) {
  hitrec rec;
  int hit = sphere_hit(s, mk(o[0], o[1], o[2]), mk(d[0], d[1], d[2]), tmin, tmax, &rec);
  if (hit) {
    rec_out[0] = rec.p.x, rec_out[1] = rec.p.y, rec_out[2] = rec.p.z;
    rec_out[3] = rec.normal.x, rec_out[4] = rec.normal.y, rec_out[5] = rec.normal.z;
    rec_out[6] = rec.t, rec_out[7] = rec.front_face;
  }
  return hit;
}

/* hittable_list::hit known-answer: returns hit index or -1. */
int oracle_world_hit(const rt_sphere* sph, int n, const double o[3], const double d[3],
                     double tmin, double tmax, double rec_out[8]) {
  hitrec rec;
  if (!world_hit(sph, n, mk(o[0], o[1], o[2]), mk(d[0], d[1], d[2]), tmin, tmax, &rec))
    return -1;
  rec_out[0] = rec.p.x, rec_out[1] = rec.p.y, rec_out[2] = rec.p.z;
  rec_out[3] = rec.normal.x, rec_out[4] = rec.normal.y, rec_out[5] = rec.normal.z;
  rec_out[6] = rec.t, rec_out[7] = rec.front_face;
  return rec.index;
}

/* Raw draws of both streams (RNG known-answer vectors). */
void oracle_counter_draws(uint64_t seed, uint32_t pixel, uint32_t sample, int count,
                          int32_t* out) {
  uint64_t st = oracle_stream_state(seed, pixel, sample);
  int k;
  for (k = 0; k < count; ++k) out[k] = oracle_counter_rand(&st);
}

void oracle_glibc_draws(unsigned seed, int count, int32_t* out) {
  oracle_glibc_rand g;
  int k;
  oracle_glibc_srand(&g, seed);
  for (k = 0; k < count; ++k) out[k] = oracle_glibc_next(&g);
}

/* camera() (camera.h:11-23) */
void oracle_camera_default(rt_camera* c) {
  double aspect = 16.0 / 9.0, vh = 2.0, vw = vh * aspect, focal = 1.0;
  v3 org = mk(0, 0, 0), h = mk(vw, 0, 0), v = mk(0, vh, 0);
  v3 llc = add(sub(sub(org, divs(h, 2.0)), divs(v, 2.0)), mk(0, 0, -focal));
  c->origin[0] = org.x, c->origin[1] = org.y, c->origin[2] = org.z;
  c->horizontal[0] = h.x, c->horizontal[1] = h.y, c->horizontal[2] = h.z;
  c->vertical[0] = v.x, c->vertical[1] = v.y, c->vertical[2] = v.z;
  c->lower_left[0] = llc.x, c->lower_left[1] = llc.y, c->lower_left[2] = llc.z;
}

/* Book-style look-at pinhole (extension). */
void oracle_camera_look_at(const double from[3], const double at[3], const double up[3],
                           double vfov_deg, double aspect, rt_camera* c) {
  double theta = vfov_deg * 3.1415926535897932385 / 180.0; /* raytracer.h:15-17 */
  double hh = tan(theta / 2);
  double vh = 2.0 * hh, vw = aspect * vh;
  v3 lf = mk(from[0], from[1], from[2]), la = mk(at[0], at[1], at[2]);
  v3 vup = mk(up[0], up[1], up[2]);
  v3 w = unit(sub(lf, la));
  v3 u = unit(cross3(vup, w));
  v3 v = cross3(w, u);
  v3 h = scale(vw, u), vv = scale(vh, v);
  v3 llc = sub(sub(sub(lf, divs(h, 2.0)), divs(vv, 2.0)), w);
  c->origin[0] = lf.x, c->origin[1] = lf.y, c->origin[2] = lf.z;
  c->horizontal[0] = h.x, c->horizontal[1] = h.y, c->horizontal[2] = h.z;
  c->vertical[0] = vv.x, c->vertical[1] = vv.y, c->vertical[2] = vv.z;
  c->lower_left[0] = llc.x, c->lower_left[1] = llc.y, c->lower_left[2] = llc.z;
}

/* Final random-spheres scene, diffuse only: glibc
 * srand(seed); per cell one choose draw, then x then z jitter draws. */
int oracle_scene_random_spheres(unsigned seed, rt_sphere* out, int cap) {
  oracle_glibc_rand g;
  orng r;
  int a, b, n = 0;
  oracle_glibc_srand(&g, seed);
  memset(&r, 0, sizeof r);
  r.mode = ORACLE_RNG_GLIBC;
  r.glibc = &g;
#define PUSH(X, Y, Z, R)                                        \
  do {                                                          \
    if (n < cap) {                                              \
      out[n].cx = (X), out[n].cy = (Y), out[n].cz = (Z), out[n].r = (R); \
    }                                                           \
    ++n;                                                        \
  } while (0)
  PUSH(0.0, -1000.0, 0.0, 1000.0);
  for (a = -11; a < 11; ++a) {
    for (b = -11; b < 11; ++b) {
      double choose = random_double(&r);
      double cx = a + 0.9 * random_double(&r);
      double cz = b + 0.9 * random_double(&r);
      v3 c = mk(cx, 0.2, cz);
      v3 dd = sub(c, mk(4, 0.2, 0));
      (void)choose;
      if (sqrt(dd.x * dd.x + dd.y * dd.y + dd.z * dd.z) > 0.9) PUSH(cx, 0.2, cz, 0.2);
    }
  }
  PUSH(0.0, 1.0, 0.0, 1.0);
  PUSH(-4.0, 1.0, 0.0, 1.0);
  PUSH(4.0, 1.0, 0.0, 1.0);
#undef PUSH
  return n;
}
