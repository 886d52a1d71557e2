/* Launch-tail model for C3 (final scene, 1200x800, depth 50): how long are the
 * paths the device traces (the trapped-path exit of DESIGN.md §9 applied), and
 * are the long ones predictable per pixel? A longest-first pixel order would
 * shorten the one-frame launch's drain only if they are. Analysis only.
 *   gcc -O2 -ffp-contract=off -Ioracle -o /tmp/tail_model tests/models/tail_model.c -lm -lpthread
 *   /tmp/tail_model 3000 100 */
#include "../oracle/rt_oracle.c"
#include <stdio.h>
static double Cof(const rt_sphere* s, const double o[3]) {
  double ax = o[0] - s->cx, ay = o[1] - s->cy, az = o[2] - s->cz;
  return ((ax * ax + ay * ay) + az * az) - s->r * s->r;
}
static int cmp_desc(const void* a, const void* b) {
  double x = ((const double*)a)[0], y = ((const double*)b)[0];
  return x < y ? 1 : x > y ? -1 : 0;
}
int main(int argc, char** argv) {
  rt_sphere sph[600];
  int n = oracle_scene_random_spheres(1, sph, 600);
  rt_camera cam;
  double from[3] = {13, 2, 3}, at[3] = {0, 0, 0}, up[3] = {0, 1, 0};
  oracle_camera_look_at(from, at, up, 20.0, 1200.0 / 800.0, &cam);
  rt_params p;
  memset(&p, 0, sizeof p);
  p.width = 1200, p.height = 800, p.spp = 100, p.max_depth = 50, p.seed = 0;
  oracle_bounce tr[64];
  const int NP = argc > 1 ? atoi(argv[1]) : 3000, NS = argc > 2 ? atoi(argv[2]) : 100;
  /* per pixel: [mean L, P(L >= 30), index i, j] */
  double* px = calloc((size_t)NP * 4, sizeof(double));
  int* L_all = calloc((size_t)NP * NS, sizeof(int));
  long hist[64] = {0};
  uint64_t x = 777;
  for (int k = 0; k < NP; ++k) {
    x = x * 6364136223846793005ULL + 1442695040888963407ULL;
    const int i = (int)((x >> 33) % 1200), j = (int)((x >> 13) % 800);
    double sum = 0, longc = 0;
    for (int s = 0; s < NS; ++s) {
      double col[3];
      const int len = oracle_trace_sample(sph, n, &cam, &p, i, j, s, col, tr, 64);
      int L = len;
      for (int r = 1; r < len; ++r) {
        const int h = tr[r - 1].index;
        if (h >= 0 && Cof(&sph[h], tr[r].o) == 0.0) { L = r + 1; break; }
      }
      L_all[(size_t)k * NS + s] = L;
      hist[L < 63 ? L : 63]++;
      sum += L;
      longc += L >= 30;
    }
    px[4 * k] = sum / NS, px[4 * k + 1] = longc / NS, px[4 * k + 2] = i, px[4 * k + 3] = j;
  }
  if (argc > 3) {  /* per (pixel, sample) traced rays, pixel-major, + the pixels' (i, j) */
    FILE* f = fopen(argv[3], "wb");
    fwrite(L_all, sizeof(int), (size_t)NP * NS, f);
    for (int k = 0; k < NP; ++k) {
      const int ij[2] = {(int)px[4 * k + 2], (int)px[4 * k + 3]};
      fwrite(ij, sizeof(int), 2, f);
    }
    fclose(f);
  }
  long tot = (long)NP * NS, acc = 0;
  printf("{\"samples\": %ld, \"traced_L_hist\": {", tot);
  for (int L = 1; L < 64; ++L)
    if (hist[L]) printf("%s\"%d\": %ld", acc++ ? ", " : "", L, hist[L]);
  printf("}}\n");
  long ge[5] = {0};
  const int th[5] = {10, 20, 30, 40, 51};
  for (long q = 0; q < tot; ++q)
    for (int t = 0; t < 5; ++t) ge[t] += L_all[q] >= th[t];
  printf("{\"P(L>=10,20,30,40,51)\": [%.5f, %.5f, %.5f, %.5f, %.5f]}\n", (double)ge[0] / tot,
         (double)ge[1] / tot, (double)ge[2] / tot, (double)ge[3] / tot, (double)ge[4] / tot);
  /* predictability: pixels split in two halves of samples; rank pixels by the
   * first half's mean L, and count the second half's long samples (L >= 30)
   * in the last 10 / 20% of a longest-first order against the natural order */
  double* rk = calloc((size_t)NP * 2, sizeof(double));
  for (int k = 0; k < NP; ++k) {
    double m = 0;
    for (int s = 0; s < NS / 2; ++s) m += L_all[(size_t)k * NS + s];
    rk[2 * k] = m, rk[2 * k + 1] = k;
  }
  qsort(rk, NP, 2 * sizeof(double), cmp_desc);
  for (int frac = 10; frac <= 20; frac += 10) {
    const int from_k = NP - NP * frac / 100;
    long lj = 0, nat = 0, all = 0;
    for (int r = 0; r < NP; ++r) {
      const int k = (int)rk[2 * r + 1];
      for (int s = NS / 2; s < NS; ++s) {
        const int L = L_all[(size_t)k * NS + s];
        if (L >= 30) { all++; if (r >= from_k) lj++; }
      }
    }
    /* natural order: the pixels' reference order (rows top to bottom) */
    double* nat_k = calloc((size_t)NP * 2, sizeof(double));
    for (int k = 0; k < NP; ++k) nat_k[2 * k] = -( (799 - px[4 * k + 3]) * 1200 + px[4 * k + 2]), nat_k[2 * k + 1] = k;
    qsort(nat_k, NP, 2 * sizeof(double), cmp_desc);
    for (int r = from_k; r < NP; ++r) {
      const int k = (int)nat_k[2 * r + 1];
      for (int s = NS / 2; s < NS; ++s) nat += L_all[(size_t)k * NS + s] >= 30;
    }
    free(nat_k);
    printf("{\"last_%d%%_of_pixels\": {\"long_samples_total\": %ld, \"longest_first_order\": %ld, "
           "\"reference_order\": %ld}}\n", frac, all, lj, nat);
  }
  return 0;
}
