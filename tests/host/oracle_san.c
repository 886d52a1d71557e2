/* The oracle's C restatement (oracle/rt_oracle.c) under AddressSanitizer /
 * UndefinedBehaviorSanitizer (UBSan is what would have flagged
 * the int overflow of random.h:7): small frames in both RNG modes, threaded
 * and serial, and hittable_list::hit on edge rays (zero, NaN and huge
 * directions, origins on / inside spheres). Prints "ok" on success.
 * Built by tests/test_sanitizers.py with -fsanitize=address,undefined. */
#include <math.h>
#include <stdio.h>
#include <string.h>

#include "../../include/rt.h"

int oracle_render(const rt_sphere*, int, const rt_camera*, const rt_params*, int, int, double*,
                  unsigned char*, unsigned long long*);
int oracle_world_hit(const rt_sphere*, int, const double*, const double*, double, double, double*);
int oracle_scene_random_spheres(unsigned, rt_sphere*, int);
void oracle_camera_default(rt_camera*);
void oracle_camera_look_at(const double*, const double*, const double*, double, double, rt_camera*);
int oracle_render_mat(const rt_sphere*, const rt_material*, int, const rt_camera_lens*,
                      const rt_params*, int, double*, unsigned long long*);
int oracle_scene_book_final(unsigned, rt_sphere*, rt_material*, int);
void oracle_camera_look_at_lens(const double*, const double*, const double*, double, double,
                                double, double, rt_camera_lens*);

static double acc1[40 * 24 * 3], acc2[40 * 24 * 3];
static unsigned char rgb[40 * 24 * 3];

int main(void) {
  rt_sphere two[2] = {{0, 0, -1, 0.5}, {0, -100.5, 0, 100}};
  static rt_sphere fin[1024];
  const int nf = oracle_scene_random_spheres(1, fin, 1024);
  rt_camera cd, cl;
  const double from[3] = {13, 2, 3}, at[3] = {0, 0, 0}, up[3] = {0, 1, 0};
  unsigned long long rays = 0;
  int bad = 0;
  oracle_camera_default(&cd);
  oracle_camera_look_at(from, at, up, 20.0, 40.0 / 24.0, &cl);
  rt_params p = {40, 24, 3, 50, 0, 0, 1, 0};
  /* glibc stream (serial) and counter stream (1 and 4 threads) */
  bad |= oracle_render(two, 2, &cd, &p, 1, 1, acc1, rgb, &rays) != 0;
  bad |= oracle_render(two, 2, &cd, &p, 0, 1, acc1, rgb, &rays) != 0;
  bad |= oracle_render(two, 2, &cd, &p, 0, 4, acc2, rgb, &rays) != 0;
  bad |= memcmp(acc1, acc2, sizeof acc1) != 0;
  p.spp = 1;
  bad |= oracle_render(fin, nf, &cl, &p, 0, 3, acc1, rgb, &rays) != 0;
  p.max_depth = -1;
  bad |= oracle_render(fin, nf, &cl, &p, 0, 2, acc1, rgb, &rays) != 0;
  p.max_depth = 0, p.row_offset = 5, p.row_stride = 7;
  bad |= oracle_render(fin, nf, &cl, &p, 0, 2, acc1, rgb, &rays) != 0;
  {
    const double o[6][3] = {{0, 0, 0}, {0, 0, -1}, {0, 0, -0.5}, {1e300, 0, 0}, {0, 0, 0}, {0, 0.5, -1}};
    const double d[6][3] = {{0, 0, 0}, {1, 0, 0}, {0, 0, -1}, {-1, 0, 0}, {NAN, 0, 1}, {1e200, 1e-200, 0}};
    double rec[8];
    for (int k = 0; k < 6; ++k) {
      (void)oracle_world_hit(two, 2, o[k], d[k], 0.0, INFINITY, rec);
      (void)oracle_world_hit(fin, nf, o[k], d[k], 0.0, INFINITY, rec);
    }
  }
  { /* the materials extension (rt_oracle_mat.c): book scene, lens, depth edges */
    static rt_sphere bs[600];
    static rt_material bm[600];
    rt_camera_lens lc;
    const int nb = oracle_scene_book_final(1, bs, bm, 600);
    oracle_camera_look_at_lens(from, at, up, 20.0, 40.0 / 24.0, 0.1, 10.0, &lc);
    p.max_depth = 50, p.row_offset = 0, p.row_stride = 1, p.spp = 2;
    bad |= oracle_render_mat(bs, bm, nb, &lc, &p, 3, acc1, &rays) != 0;
    bad |= oracle_render_mat(bs, bm, nb, &lc, &p, 1, acc2, &rays) != 0;
    bad |= memcmp(acc1, acc2, sizeof acc1) != 0;
    p.max_depth = 4096, p.spp = 1;
    bad |= oracle_render_mat(bs, bm, nb, &lc, &p, 2, acc1, &rays) != 0;
    p.max_depth = 4097;
    bad |= oracle_render_mat(bs, bm, nb, &lc, &p, 2, acc1, &rays) != RT_E_INVALID;
  }
  printf(bad ? "FAIL\n" : "ok\n");
  return bad;
}
