// psrt_ablate.h — section ablation for the census.
// MEASUREMENT BUILDS ONLY: psrt_kernels.hip / psrt_mat.hip include this file
// only when PSRT_ABLATE / PSRT_MAT_ABLATE is non-zero (scripts/build_variants.py
// PSRT_ABLATE=<id>); the product build expands every hook to nothing, so the
// shipped kernels' ISA does not depend on this file.
//
// A hook runs its section a second time on copies of the section's state and
// sinks the copy's results through an empty asm, so PMC SQ_INSTS_VALU and the
// kernel time grow by that section's cost. Each hook names the kernel's own
// locals: it is pasted at its site and compiles only there.
// Included inside the kernel file's namespace.
#pragma once

template <class T>
__device__ __forceinline__ void ablate_sink(T v) {
  asm volatile("" ::"v"(v));
}
template <class T>
__device__ __forceinline__ T ablate_launder(T v) {
  asm volatile("" : "+v"(v));
  return v;
}

// ---- psrt_trace (PSRT_ABLATE = section id) ----------------------------------

#if PSRT_ABLATE == 1  // hit_quick, whole
#define PSRT_ABLATE_HIT_QUICK()                                                            \
  {                                                                                        \
    double bt2;                                                                            \
    int bi2;                                                                               \
    bool tr2;                                                                              \
    CullStatsT<false> cs2{};                                                               \
    float t02;                                                                             \
    const bool r2 = hit_quick(geo, sv, a.n, bv, hint, ox, oy, oz, dx, dy, dz, A, bt2, bi2, \
                              cs2, clk, tr2, q, gc, lbig, t02);                            \
    ablate_sink(bt2), ablate_sink(bi2), ablate_sink(tr2), ablate_sink(r2);                 \
  }
#endif

#if PSRT_ABLATE == 2  // the batched BVH walk
#define PSRT_ABLATE_WALK()                                                                 \
  {                                                                                        \
    double bt2 = pbt;                                                                      \
    int bi2 = pbi, n2 = wnode;                                                             \
    CullStatsT<false> cs2{};                                                               \
    hit_traverse<false, kLds>(bv, nodes, lleaf, sv, hint, ox, oy, oz, dx, dy, dz, A, bt2,  \
                              bi2, cs2, n2, movable ? kWalkTail : 0u, (double)wt0);        \
    ablate_sink(bt2), ablate_sink(bi2), ablate_sink(n2);                                   \
  }
#endif

#if PSRT_ABLATE == 3  // the look-ahead trials
#define PSRT_ABLATE_TRIALS()                                                               \
  {                                                                                        \
    const bool can_fill = active && !finish;                                               \
    uint64_t rng2 = rng;                                                                   \
    uint32_t a0x = q0x, a0y = q0y, a0z = q0z, a1x = q1x, a1y = q1y, a1z = q1z;             \
    bool v0 = qv0, v1 = qv1;                                                               \
    int f = 0;                                                                             \
    do {                                                                                   \
      const bool go = can_fill && !v1;                                                     \
      uint32_t z, y, x;                                                                    \
      uint64_t nxt;                                                                        \
      raw32_x3(rng2, z, y, x, nxt);                                                        \
      const bool in = in_unit_sphere_raw_f32(x, y, z);                                     \
      rng2 = go ? nxt : rng2;                                                              \
      const bool push = go && in;                                                          \
      const bool to0 = push && !v0, to1 = push && v0;                                      \
      a0x = to0 ? x : a0x, a0y = to0 ? y : a0y, a0z = to0 ? z : a0z;                       \
      a1x = to1 ? x : a1x, a1y = to1 ? y : a1y, a1z = to1 ? z : a1z;                       \
      v1 = v1 || to1;                                                                      \
      v0 = v0 || to0;                                                                      \
      ++f;                                                                                 \
    } while (f < kRngFill || (f < kRngFill + kRngExtra && __ballot(want && !v0) != 0));    \
    ablate_sink(rng2), ablate_sink(a0x), ablate_sink(a0y), ablate_sink(a0z);               \
    ablate_sink(a1x), ablate_sink(a1y), ablate_sink(a1z), ablate_sink(v0), ablate_sink(v1); \
  }
#endif

#if PSRT_ABLATE == 4  // scatter (hit record + new ray)
#define PSRT_ABLATE_SCATTER()                                                              \
  if (want && have) {                                                                      \
    const HitRec h = hit_record_of(sv.geo(hit), sv.inv(hit), t, ox, oy, oz, dx, dy, dz);   \
    double rx = pm1_raw(q0x), ry = pm1_raw(q0y), rz = pm1_raw(q0z);                        \
    if (!((rx * h.nx + ry * h.ny) + rz * h.nz > 0.0)) rx = -rx, ry = -ry, rz = -rz;        \
    const double ex = ((h.px + h.nx) + rx) - h.px;                                         \
    const double ey = ((h.py + h.ny) + ry) - h.py;                                         \
    const double ez = ((h.pz + h.nz) + rz) - h.pz;                                         \
    ablate_sink((ex * ex + ey * ey) + ez * ez), ablate_sink(h.px), ablate_sink(h.py);      \
    ablate_sink(h.pz);                                                                     \
  }
#endif

#if PSRT_ABLATE == 5  // refill per-lane setup (stream, u, v, get_ray)
#define PSRT_ABLATE_REFILL()                                                               \
  {                                                                                        \
    uint64_t r2 = splitmix64((((uint64_t)pix) << 32 | (uint64_t)s) ^ rc.seedmix[f]);        \
    const double xu2 = (double)i + random_double(r2), xv2 = (double)j + random_double(r2); \
    const double u2 = div_by(xu2, rc.wm1, rc.rwm1), v2 = div_by(xv2, rc.hm1, rc.rhm1);     \
    const double* c2 = rc.cam;                                                             \
    const double ex = ((c2[3] + u2 * c2[6]) + v2 * c2[9]) - c2[0];                         \
    const double ey = ((c2[4] + u2 * c2[7]) + v2 * c2[10]) - c2[1];                        \
    const double ez = ((c2[5] + u2 * c2[8]) + v2 * c2[11]) - c2[2];                        \
    ablate_sink((ex * ex + ey * ey) + ez * ez), ablate_sink(r2);                           \
  }
#endif

#if PSRT_ABLATE == 6  // hit_quick: the hint test
#define PSRT_ABLATE_HINT()                                                                 \
  {                                                                                        \
    double bt2 = __builtin_inf(), ch2;                                                     \
    int bi2 = -1;                                                                          \
    test_sphere<false>(sh, hint, ox, oy, oz, dx, dy, dz, A, bt2, bi2, float4{}, pr, &ch2); \
    ablate_sink(bt2), ablate_sink(bi2), ablate_sink(ch2);                                  \
  }
#endif

#if PSRT_ABLATE == 7  // hit_quick: the big spheres
#define PSRT_ABLATE_BIG()                                                                  \
  {                                                                                        \
    double bt2 = bt;                                                                       \
    int bi2 = bi;                                                                          \
    bool f2 = false;                                                                       \
    for (int b = 0; b < bv.n_big; ++b) {                                                   \
      const int idx = lbig[b];                                                             \
      if (idx != hint)                                                                     \
        f2 |= test_sphere(sv.geo(idx), idx, ox, oy, oz, dx, dy, dz, A, bt2, bi2,           \
                          sv.g32(idx), pr);                                                \
    }                                                                                      \
    ablate_sink(bt2), ablate_sink(bi2), ablate_sink(f2);                                   \
  }
#endif

#if PSRT_ABLATE == 8  // hit_quick: the candidate list
#define PSRT_ABLATE_LIST()                                                                 \
  {                                                                                        \
    double bt2 = bt;                                                                       \
    int bi2 = bi;                                                                          \
    bool f2 = false;                                                                       \
    uint64_t lo2 = lo, hi2 = hi;                                                           \
    for (int e = 0; e < cnt; ++e) {                                                        \
      lo2 = (lo2 >> 16) | (hi2 << 48);                                                     \
      hi2 >>= 16;                                                                          \
      const int idx = (int)(lo2 & 0xFFFFu);                                                \
      if (idx == hint) continue;                                                           \
      f2 |= test_sphere(sv.geo(idx), idx, ox, oy, oz, dx, dy, dz, A, bt2, bi2,             \
                        sv.g32(idx), pr);                                                  \
    }                                                                                      \
    ablate_sink(bt2), ablate_sink(bi2), ablate_sink(f2);                                   \
  }
#endif

// ---- psrt_trace_mat (PSRT_MAT_ABLATE = section id) ---------------------------

#if PSRT_MAT_ABLATE == 1  // hit_quick_m
#define PSRT_MAT_ABLATE_HIT()                                                              \
  {                                                                                        \
    double bt2;                                                                            \
    int bi2;                                                                               \
    const bool d2 = hit_quick_m<kBVH>(ntests, nroots, lgeo, a.n, bv, big_idx, gc, rec,     \
                                      ablate_launder(ox), ablate_launder(oy),              \
                                      ablate_launder(oz), ablate_launder(dx),              \
                                      ablate_launder(dy), ablate_launder(dz),              \
                                      ablate_launder(A), bt2, bi2);                        \
    ablate_sink(bt2), ablate_sink(bi2), ablate_sink(d2);                                   \
  }
#endif

#if PSRT_MAT_ABLATE == 2  // the batched walk (state copied before, re-run after)
#define PSRT_MAT_ABLATE_WALK_SAVE() \
  double bt2 = ablate_launder(pbt); \
  int bi2 = ablate_launder(pbi);
#define PSRT_MAT_ABLATE_WALK_RUN()                                                         \
  hit_walk_m(ntests, nboxes, nroots, bv, nodes, leaf_geo, leaf_idx, ablate_launder(ox),    \
             ablate_launder(oy), ablate_launder(oz), ablate_launder(dx), ablate_launder(dy), \
             ablate_launder(dz), ablate_launder(A), bt2, bi2);                             \
  ablate_sink(bt2), ablate_sink(bi2);
#endif

#if PSRT_MAT_ABLATE == 3  // the random_in_unit_sphere trial loop
#define PSRT_MAT_ABLATE_TRIALS()                       \
  {                                                    \
    uint64_t r2 = ablate_launder(rng);                 \
    uint32_t z2, y2, x2;                               \
    for (;;) {                                         \
      raw32_x3(r2, z2, y2, x2, r2);                    \
      if (in_unit_sphere_raw(x2, y2, z2)) break;       \
    }                                                  \
    ablate_sink(z2), ablate_sink(y2), ablate_sink(x2), ablate_sink(r2); \
  }
#endif

#if PSRT_MAT_ABLATE == 4  // the hit record
#define PSRT_MAT_ABLATE_RECORD()                                                           \
  {                                                                                        \
    const int bi2 = ablate_launder(bi);                                                    \
    const HitRec h2 = hit_record_of(lgeo[bi2], linv[bi2], ablate_launder(pbt),             \
                                    ablate_launder(ox), ablate_launder(oy),                \
                                    ablate_launder(oz), ablate_launder(dx),                \
                                    ablate_launder(dy), ablate_launder(dz));               \
    ablate_sink(h2.px), ablate_sink(h2.py), ablate_sink(h2.pz), ablate_sink(h2.nx),        \
        ablate_sink(h2.ny), ablate_sink(h2.nz), ablate_sink(h2.front);                     \
  }
#endif

#if PSRT_MAT_ABLATE == 5  // the refill's per-lane setup
#define PSRT_MAT_ABLATE_SETUP()                                                            \
  {                                                                                        \
    uint64_t r2;                                                                           \
    double o2x, o2y, o2z, d2x, d2y, d2z, A2;                                               \
    unsigned q2;                                                                           \
    setup(ablate_launder(su), r2, o2x, o2y, o2z, d2x, d2y, d2z, A2, q2);                   \
    ablate_sink(q2);                                                                       \
    ablate_sink(r2), ablate_sink(o2x), ablate_sink(o2y), ablate_sink(o2z),                 \
        ablate_sink(d2x), ablate_sink(d2y), ablate_sink(d2z), ablate_sink(A2);             \
  }
#endif

// ---- hook dispatch: the sites not selected by this build expand to nothing ----
#define PSRT_ABLATE_AT(site) PSRT_ABLATE_##site()
#define PSRT_MAT_ABLATE_AT(site) PSRT_MAT_ABLATE_##site()
#ifndef PSRT_ABLATE_HIT_QUICK
#define PSRT_ABLATE_HIT_QUICK()
#endif
#ifndef PSRT_ABLATE_WALK
#define PSRT_ABLATE_WALK()
#endif
#ifndef PSRT_ABLATE_TRIALS
#define PSRT_ABLATE_TRIALS()
#endif
#ifndef PSRT_ABLATE_SCATTER
#define PSRT_ABLATE_SCATTER()
#endif
#ifndef PSRT_ABLATE_REFILL
#define PSRT_ABLATE_REFILL()
#endif
#ifndef PSRT_ABLATE_HINT
#define PSRT_ABLATE_HINT()
#endif
#ifndef PSRT_ABLATE_BIG
#define PSRT_ABLATE_BIG()
#endif
#ifndef PSRT_ABLATE_LIST
#define PSRT_ABLATE_LIST()
#endif
#ifndef PSRT_MAT_ABLATE_HIT
#define PSRT_MAT_ABLATE_HIT()
#endif
#ifndef PSRT_MAT_ABLATE_WALK_SAVE
#define PSRT_MAT_ABLATE_WALK_SAVE()
#define PSRT_MAT_ABLATE_WALK_RUN()
#endif
#ifndef PSRT_MAT_ABLATE_TRIALS
#define PSRT_MAT_ABLATE_TRIALS()
#endif
#ifndef PSRT_MAT_ABLATE_RECORD
#define PSRT_MAT_ABLATE_RECORD()
#endif
#ifndef PSRT_MAT_ABLATE_SETUP
#define PSRT_MAT_ABLATE_SETUP()
#endif
