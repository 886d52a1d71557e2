/* Rays of sampled book-scene paths (the C restatement of the material path,
   oracle/rt_oracle_mat.c), for tests/models/mat_walk_model.cc: per ray o, d, t, hit
   index, bounce. Build and run: see mat_walk_model.cc. */
#include "rt_oracle_mat.c" /* -I oracle */
#include <stdio.h>
int main(int argc, char** argv) {
  long N = argc > 1 ? atol(argv[1]) : 20000;
  rt_sphere sph[600]; rt_material mats[600];
  int n = oracle_scene_book_final(1, sph, mats, 600);
  rt_camera_lens cm;
  double from[3] = {13, 2, 3}, at[3] = {0, 0, 0}, up[3] = {0, 1, 0};
  oracle_camera_look_at_lens(from, at, up, 20.0, 1.5, 0.1, 10.0, &cm);
  FILE* f = fopen(argc > 2 ? argv[2] : "mat_rays.bin", "wb");
  uint64_t x = 777;
  long nr = 0;
  for (long it = 0; it < N; ++it) {
    x = x * 6364136223846793005ULL + 1442695040888963407ULL;
    int i = (x >> 33) % 1200, j = (x >> 13) % 800, s = (x >> 50) % 10;
    uint64_t st = oracle_stream_state(0, (uint32_t)(j * 1200 + i), (uint32_t)s);
    double u = ((double)i + rd(&st)) / 1199.0, v = ((double)j + rd(&st)) / 799.0;
    m3 rdk = in_unit_disk(&st);
    double rx = cm.lens_radius * rdk.x, ry = cm.lens_radius * rdk.y;
    m3 off = add3(mul3(rx, mk3(cm.u[0], cm.u[1], cm.u[2])), mul3(ry, mk3(cm.v[0], cm.v[1], cm.v[2])));
    m3 org = mk3(cm.base.origin[0], cm.base.origin[1], cm.base.origin[2]);
    m3 o = add3(org, off);
    m3 d = sub3(sub3(add3(add3(mk3(cm.base.lower_left[0], cm.base.lower_left[1], cm.base.lower_left[2]),
                                mul3(u, mk3(cm.base.horizontal[0], cm.base.horizontal[1], cm.base.horizontal[2]))),
                           mul3(v, mk3(cm.base.vertical[0], cm.base.vertical[1], cm.base.vertical[2]))), org), off);
    for (int depth = 50, k = 0; depth > 0; --depth, ++k) {
      mrec rec;
      int hit = world_hit_m(sph, n, o, d, 0.001, &rec);
      double w[8] = {o.x, o.y, o.z, d.x, d.y, d.z, hit ? rec.t : -1.0, (double)(hit ? rec.idx : -1)};
      double kk = k;
      fwrite(w, sizeof w, 1, f); fwrite(&kk, 8, 1, f); ++nr;
      if (!hit) break;
      const rt_material* m = &mats[rec.idx];
      m3 dir; int ok = 1;
      if (m->kind == RT_MAT_LAMBERTIAN) {
        dir = add3(rec.n, unitm(in_unit_sphere(&st)));
        if (fabs(dir.x) < 1e-8 && fabs(dir.y) < 1e-8 && fabs(dir.z) < 1e-8) dir = rec.n;
      } else if (m->kind == RT_MAT_METAL) {
        double fz = m->fuzz < 1 ? m->fuzz : 1;
        dir = add3(reflectm(unitm(d), rec.n), mul3(fz, in_unit_sphere(&st)));
        ok = dotm(dir, rec.n) > 0;
      } else {
        double ratio = rec.front ? (1.0 / m->ir) : m->ir;
        m3 ud = unitm(d);
        double ct = fmin(dotm(neg3(ud), rec.n), 1.0), stt = sqrt(1.0 - ct * ct);
        if (ratio * stt > 1.0 || reflectance(ct, ratio) > rd(&st)) dir = reflectm(ud, rec.n);
        else dir = refractm(ud, rec.n, ratio);
      }
      if (!ok) break;
      o = rec.p; d = dir;
    }
  }
  fclose(f);
  printf("rays %ld n %d\n", nr, n);
  return 0;
}
