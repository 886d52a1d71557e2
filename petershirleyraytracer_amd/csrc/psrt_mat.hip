// psrt_mat.hip — the material integrator.
//
// A kernel variant of its own: the reference integrator (psrt_trace,
// psrt_kernels.hip) keeps its code, bits and RNG consumption. This one traces
// the book's continuation of the reference (Ray Tracing in One Weekend v3.2,
// ch. 9-13; DESIGN.md §14 restates it):
//
//   psrt_trace_mat   persistent lanes, one camera sample per work unit:
//                    thin-lens get_ray, then ray_color as a bounce loop —
//                    world.hit(r, 0.001, inf) (hittable_list.cc:3-20 /
//                    sphere.cc:3-40 over [tmin, closest]), lambertian / metal /
//                    dielectric scatter; a finished sample stores its colour
//                    (3 doubles) in unit order.
//   psrt_reduce_rgb  pixel_color += sample in sample order (main.cc:77-84),
//                    then write_color (color.h:8-24) on the last chunk.
//
// The recursion's product attenuation * ray_color(...) is taken innermost
// first, so it is formed when the path ends: each lane keeps the indices of
// the attenuating hits of its path in a scratch column (MatArgs::path;
// dielectric hits attenuate by exactly 1 and are not kept), and multiplies
// the sky colour by their albedos in reverse.
//
// Culling: the BVH (psrt_bvh.h) bounds every sphere with a root in
// [0, closest], so it bounds [0.001, closest] too; each lane walks it on its
// own (stackless skip links). Ties and the root rule are the reference's:
// the lexicographic minimum of (t, -index), t = near root if >= tmin, else
// far root if >= tmin. Rays the BVH cannot bound take the linear scan.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/rt.h"
#include "psrt_device.h"
#include "psrt_geom.h"
#include "psrt_kernels.h"

namespace psrt {
namespace {

constexpr double kTmin = 0.001;
  // the book's world.hit(r, 0.001, infinity)
// Wave issue priorities (as psrt_trace): the latency-bound
// sections (the grid query and list tests, the batched walk) issue first,
// the dependency-light scatter fills the gaps. Book scene: 2.58 -> 2.49 ms
// per frame (r04, profiles/r04_mat/ab.txt); two BVH nodes per walk trip
// were slower here (2.72 ms) and are not used.
constexpr int kMatHitPrio = 2;
constexpr int kMatWalkPrio = 3;

// Section ablation for the census: measurement builds only
// (PSRT_MAT_ABLATE = section id, psrt_ablate.h: 1 hit_quick_m, 2 the batched
// walk, 3 the random_in_unit_sphere trial loop, 4 the hit record, 5 the
// refill's per-lane setup); in the product build every hook is empty.
#ifndef PSRT_MAT_ABLATE
#define PSRT_MAT_ABLATE 0
#endif
#if PSRT_MAT_ABLATE
#include "psrt_ablate.h"
#else
#define PSRT_MAT_ABLATE_AT(site)
#endif

__device__ __forceinline__ unsigned div_fast(unsigned n, const FastDiv& f) {
  const unsigned t = __umulhi(f.m, n);
  return (t + ((n - t) >> f.sh1)) >> f.sh2;
}

__device__ __forceinline__ unsigned lanes_below(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
}

// random_double(-1, 1) (random.h:10-14): min + (max - min) * random_double()
__device__ __forceinline__ double pm1(uint64_t& rng) { return -1.0 + 2.0 * random_double(rng); }

// Sphere / box test counters of the counting variant (RT_FLAG_CULL_STATS,
// kCount); in the timed kernel they fold away.
template <bool kOn>
struct TestCount {
  unsigned long long v = 0;
  __device__ __forceinline__ void add(unsigned x) {
    if constexpr (kOn) v += x;
  }
};

// sphere.cc:6-31 over [tmin, bt], then the (t, index) rule. In ascending
// index order from bt = inf this is the reference's scan exactly (NaN
// included: a NaN root passes both range tests, as there).
__device__ __forceinline__ void test_sphere_m(const double4 s, int idx, double ox, double oy,
                                              double oz, double dx, double dy, double dz, double A,
                                              double& bt, int& bi) {
  const double ax = ox - s.x, ay = oy - s.y, az = oz - s.z;
  const double hb = (dx * ax + dy * ay) + dz * az;
  const double c = ((ax * ax + ay * ay) + az * az) - s.w;
  const double disc = hb * hb - A * c;
  if (disc < 0.0) return;
  const double sq = sqrt_f64(disc);
  double t = (-hb - sq) / A;
  if (t < kTmin || t > bt) {
    t = (-hb + sq) / A;
    if (t < kTmin || t > bt) return;
  }
  if (t < bt || idx > bi) {  // equal t: the later index wins (sphere.cc:26 accepts t == tmax)
    bt = t;
    bi = idx;
  }
}

// hittable_list::hit(r, 0.001, inf) for one lane, cheap part: the big
// spheres, then the point-location grid for the segment [o, o + bt d] (as
// psrt_trace's hit_quick: a sphere with an accepted root t <= bt has its hit
// point on that segment and inside its padded box, hence in a cell the segment
// crosses; tmin = 0.001 only removes roots). Returns true when the closest hit
// is decided (bt, bi); false when the BVH must be walked from (bt, bi).
template <bool kBVH, bool kCount>
__device__ __forceinline__ bool hit_quick_m(TestCount<kCount>& nt, TestCount<kCount>& nr,
                                            const double4* __restrict__ geo,
                                            int n, const BvhView& bv,
                                            const int* __restrict__ big_idx, const GridC& gc,
                                            uint4 rec, double ox, double oy, double oz, double dx,
                                            double dy, double dz, double A, double& bt, int& bi) {
  bt = __builtin_inf();
  bi = -1;
  const double am = __builtin_fmax(__builtin_fabs(ox),
                                   __builtin_fmax(__builtin_fabs(oy), __builtin_fabs(oz)));
  // unbounded arithmetic, no BVH, or an origin beyond 2^9 S (where the
  // reference's roots may err by more than the pad, psrt_trace hit_quick):
  // the reference scan, verbatim
  if (!kBVH || !(A > 0.0 && A < 1e200) || !(am * 0.125 <= gc.r_check)) {
    for (int i = 0; i < n; ++i) test_sphere_m(geo[i], i, ox, oy, oz, dx, dy, dz, A, bt, bi);
    nt.add((unsigned)n);
    return true;
  }
  for (int b = 0; b < bv.n_big; ++b) {
    const int idx = big_idx[b];
    test_sphere_m(geo[idx], idx, ox, oy, oz, dx, dy, dz, A, bt, bi);
  }
  nt.add((unsigned)bv.n_big);
  // a camera ray with its pixel's candidate list (psrt_mat_camera_lists): the
  // listed BVH spheres are every one a ray of the pixel can hit
  const unsigned ncand = rec.x & 0xFFFFu;
  if (ncand != kCamOverflow) {
    uint64_t lo = rec.x | (uint64_t)rec.y << 32, hi = rec.z | (uint64_t)rec.w << 32;
    for (unsigned e = 0; e < ncand; ++e) {
      lo = (lo >> 16) | (hi << 48);
      hi >>= 16;
      const int idx = (int)(lo & 0xFFFFu);
      test_sphere_m(geo[idx], idx, ox, oy, oz, dx, dy, dz, A, bt, bi);
    }
    nt.add(ncand);
    return true;
  }
  // FP32 grid query, exact within 256 S (psrt_trace hit_quick)
  const double rg = 4.0 * gc.r_check;
  const int cell = (am <= rg && (bt * bt) * A <= rg * rg)
                       ? grid_locate(gc, ox, oy, oz, dx, dy, dz, bt) : kGridNone;
  if (cell == kGridOutside) return true;  // no BVH sphere in [0, bt]
  if (cell >= 0) {
    const int e0 = bv.cell_start[cell], e1 = bv.cell_start[cell + 1];
    for (int e = e0; e < e1; ++e) {
      const int idx = bv.cell_items[e];
      test_sphere_m(geo[idx], idx, ox, oy, oz, dx, dy, dz, A, bt, bi);
    }
    nt.add((unsigned)(e1 - e0));
    return true;
  }
  // far origin: the segment [0, bt] against the padded root box (FP64)
  if (!(am <= bv.r_check)) {
    nr.add(1u);
    if (root_box_entry(bv, ox, oy, oz, dx, dy, dz, bt) < 0.0) return true;
  }
  return false;
}

// The BVH walk (stackless skip links) continuing from hit_quick_m's (bt, bi).
template <bool kCount>
__device__ __forceinline__ void hit_walk_m(TestCount<kCount>& nt, TestCount<kCount>& nb,
                                           TestCount<kCount>& nr,
                                           const BvhView& bv, const float4* __restrict__ nodes,
                                           const double4* __restrict__ leaf_geo,
                                           const int* __restrict__ leaf_idx, double ox, double oy,
                                           double oz, double dx, double dy, double dz, double A,
                                           double& bt, int& bi) {
  const double am = __builtin_fmax(__builtin_fabs(ox),
                                   __builtin_fmax(__builtin_fabs(oy), __builtin_fabs(oz)));
  // Far origins are re-based at their root-box entry (as hit_traverse): the
  // FP32 slab test then sees coordinates of the scene's scale (hit_quick_m
  // has shown the entry exists)
  double t0 = 0.0;
  if (!(am <= bv.r_check)) {
    nr.add(1u);
    t0 = __builtin_fmax(0.0, root_box_entry(bv, ox, oy, oz, dx, dy, dz, bt));
  }
  const float fox = (float)(ox + t0 * dx), foy = (float)(oy + t0 * dy), foz = (float)(oz + t0 * dz);
  const float ix = safe_inv((float)dx), iy = safe_inv((float)dy), iz = safe_inv((float)dz);
  const float oix = fox * ix, oiy = foy * iy, oiz = foz * iz;
  const float tlo = -(float)t0 * 1.00000048f;
  float tmax = tmax_up(bt - t0);
  // While-while (Aila & Laine 2009): a lane that reaches a leaf holds it
  // until every lane of the wave holds one or is done; the held leaves' FP64
  // tests then run together instead of once per trip in which any lane has one.
  int node = bv.walk0;  // the root is not tested (psrt_kernels.h BvhView::walk0)
  for (;;) {
    int leaf = -1;
    while (node < bv.n_nodes && leaf < 0) {
      const float4 n0 = nodes[2 * node], n1 = nodes[2 * node + 1];
      const int skip = __float_as_int(n1.z), lf = __float_as_int(n1.w);
      nb.add(1u);
      if (!slab_hit(n0, n1, ix, iy, iz, oix, oiy, oiz, tlo, tmax)) {
        node = skip;
      } else if (lf < 0) {
        ++node;  // interior hit: DFS order continues at node + 1
      } else {
        leaf = lf;
        node = skip;
      }
    }
    if (leaf < 0) break;
    const int first = leaf >> 8, cnt = leaf & 255;
    for (int k = first; k < first + cnt; ++k)
      test_sphere_m(leaf_geo[k], leaf_idx[k], ox, oy, oz, dx, dy, dz, A, bt, bi);
    nt.add((unsigned)cnt);
    tmax = tmax_up(bt - t0);
  }
}

// Schlick's approximation (book ch. 10.4), pow(x, 5) as (x*x)*(x*x)*x
__device__ __forceinline__ double reflectance(double cosine, double ref) {
  double r0 = (1.0 - ref) / (1.0 + ref);
  r0 = r0 * r0;
  const double x = 1.0 - cosine, x2 = x * x;
  return r0 + (1.0 - r0) * ((x2 * x2) * x);
}

}  // namespace

template <bool kBVH, bool kLds, bool kCount>
__global__ __launch_bounds__(kMatBlock, kMatWaves) void psrt_trace_mat(const double4* __restrict__ geo,
                                                            const double* __restrict__ inv_r,
                                                            double* __restrict__ rgb, MatArgs a,
                                                            BvhView bv) {
  const unsigned lane = __lane_id();
  const uint64_t total = a.total_units;
  int* const path = a.path + (size_t)blockIdx.x * kMatBlock + threadIdx.x;
  const size_t ps = a.path_stride;
  // kLds: the scene in dynamic LDS (mat_lds_layout): the walk's dependent node
  // loads and every per-hit lookup (sphere, 1/r, material) see LDS latency
  // instead of L1 / L2 latency
  extern __shared__ __attribute__((aligned(16))) unsigned char s_dyn[];
  const float4* __restrict__ nodes = bv.nodes;
  const double4* __restrict__ leaf_geo = bv.leaf_geo;
  const int* __restrict__ leaf_idx = bv.leaf_idx;
  const int* __restrict__ big_idx = bv.big_idx;
  const double4* __restrict__ lgeo = geo;
  const double* __restrict__ linv = inv_r;
  const double4* __restrict__ lmat = nullptr;  // kLds: {albedo, fuzz (metal) / ir (dielectric)}
  const int* __restrict__ lkind = nullptr;
  if constexpr (kLds) {
    const MatLdsLayout lay = mat_lds_layout(a.n, bv.n_nodes, bv.n_leaf, bv.n_big);
    float4* const sn = (float4*)(s_dyn + lay.nodes);
    double4* const slg = (double4*)(s_dyn + lay.leaf_geo);
    double4* const sg = (double4*)(s_dyn + lay.geo);
    double4* const sm = (double4*)(s_dyn + lay.mat);
    double* const sv = (double*)(s_dyn + lay.inv);
    int* const sli = (int*)(s_dyn + lay.leaf_idx);
    int* const sk = (int*)(s_dyn + lay.kind);
    int* const sb = (int*)(s_dyn + lay.big);
    for (int e = threadIdx.x; e < 2 * (bv.n_nodes + 1); e += kMatBlock) sn[e] = bv.nodes[e];
    for (int e = threadIdx.x; e < bv.n_leaf; e += kMatBlock) slg[e] = bv.leaf_geo[e], sli[e] = bv.leaf_idx[e];
    for (int e = threadIdx.x; e < a.n; e += kMatBlock) {
      const DevMaterial& m = a.mats[e];
      sg[e] = geo[e];
      sv[e] = inv_r[e];
      sm[e] = make_double4(m.albedo[0], m.albedo[1], m.albedo[2],
                           m.kind == RT_MAT_METAL ? m.fuzz : m.ir);
      sk[e] = m.kind;
    }
    for (int e = threadIdx.x; e < bv.n_big; e += kMatBlock) sb[e] = bv.big_idx[e];
    __syncthreads();
    nodes = sn, leaf_geo = slg, leaf_idx = sli, big_idx = sb;
    lgeo = sg, linv = sv, lmat = sm, lkind = sk;
  }
  // the grid constants hit_quick_m reads, in LDS (re-read per use, as psrt_trace)
  __shared__ GridC s_gc;
  if (threadIdx.x == 0) s_gc = grid_consts(bv);
  __syncthreads();
  // material of sphere i: kind, albedo, fuzz / ir
  constexpr bool kLm = kLds;
  auto mat_kind = [&](int i) { return kLm ? lkind[i] : a.mats[i].kind; };
  auto mat_albedo = [&](int i, double& r, double& g, double& b) {
    if constexpr (kLm) {
      const double4 m = lmat[i];
      r = m.x, g = m.y, b = m.z;
    } else {
      r = a.mats[i].albedo[0], g = a.mats[i].albedo[1], b = a.mats[i].albedo[2];
    }
  };
  auto mat_fuzz = [&](int i) { return kLm ? lmat[i].w : a.mats[i].fuzz; };
  auto mat_ir = [&](int i) { return kLm ? lmat[i].w : a.mats[i].ir; };

  // the refill's per-lane setup of unit su_: its stream, main.cc:80-81 and
  // the thin-lens get_ray (book ch. 12)
  auto setup = [&](unsigned su_, uint64_t& rng_, double& ox_, double& oy_, double& oz_,
                   double& dx_, double& dy_, double& dz_, double& A_, unsigned& pq_) {
    unsigned q = div_fast(su_, a.div_s);  // f * pixels + pixel (frame-major units)
    const unsigned sl = su_ - q * a.div_s.d;
    unsigned f = 0;
    if (a.frames > 1) {
      f = div_fast(q, a.div_p);
      q -= f * a.div_p.d;
    }
    pq_ = q;
    const unsigned row_k = div_fast(q, a.div_w);
    const unsigned i = q - row_k * a.div_w.d;
    const int j = (a.height - 1) - (a.row_offset + (int)row_k * a.row_stride);
    const unsigned pix = (unsigned)j * (unsigned)a.width + i;
    const unsigned s = (unsigned)a.s_begin + sl;
    rng_ = splitmix64((((uint64_t)pix) << 32 | (uint64_t)s) ^ a.seedmix[f]);
    // main.cc:80-81
    const double u = ((double)i + random_double(rng_)) / (double)(a.width - 1);
    const double v = ((double)j + random_double(rng_)) / (double)(a.height - 1);
    // thin lens (book ch. 12): rd = lens_radius * random_in_unit_disk()
    // (vec3(random_double(-1,1), random_double(-1,1), 0): draws y, x)
    double px, py;
    for (;;) {
      py = pm1(rng_);
      px = pm1(rng_);
      if (!((px * px + py * py) + 0.0 * 0.0 >= 1.0)) break;
    }
    const double rx = a.lens_radius * px, ry = a.lens_radius * py;
    const double fx = a.lu[0] * rx + a.lv[0] * ry;
    const double fy = a.lu[1] * rx + a.lv[1] * ry;
    const double fz = a.lu[2] * rx + a.lv[2] * ry;
    ox_ = a.org[0] + fx;
    oy_ = a.org[1] + fy;
    oz_ = a.org[2] + fz;
    dx_ = (((a.llc[0] + u * a.hor[0]) + v * a.ver[0]) - a.org[0]) - fx;
    dy_ = (((a.llc[1] + u * a.hor[1]) + v * a.ver[1]) - a.org[1]) - fy;
    dz_ = (((a.llc[2] + u * a.hor[2]) + v * a.ver[2]) - a.org[2]) - fz;
    A_ = (dx_ * dx_ + dy_ * dy_) + dz_ * dz_;
  };

  uint64_t win_base = 0;
  unsigned win_left = 0;
  unsigned qnext = 0;  // heads found past the end of the work (this block's first)
  bool exhausted = false;

  bool active = false;
  double ox = 0, oy = 0, oz = 0, dx = 0, dy = 0, dz = 0, A = 0;
  int k = 0, np = 0;  // hits so far / attenuating hits kept in `path`
  uint64_t rng = 0;   // the sample's stream: position of its next draw
  unsigned su = 0;
  unsigned pq = 0;    // the sample's pixel within the shard (camera list index)
  unsigned long long rays = 0;
  // Rays the grid cannot decide park (pending) with their partial (pbt, pbi)
  // and are walked together once a.batch lanes wait or nothing else can move
  // (psrt_trace's batched walk): the walk then runs for many lanes at once.
  bool pending = false;
  int pbi = -1;
  double pbt = 0.0;
  // RT_FLAG_CULL_STATS: executed FP64 sphere tests (every test here is a full
  // one: no pre-reject), FP32 box tests, FP64 root-box tests
  TestCount<kCount> ntests, nboxes, nroots;

  for (;;) {
    // ---- refill idle lanes from the wave's window (ballot + mbcnt) ----
    const uint64_t need = __ballot(!active);
    if (need != 0 && !exhausted) {
      const unsigned cnt = (unsigned)__popcll(need), rank = lanes_below(need);
      uint64_t nb = 0;
      bool fresh = false;
      if (cnt > win_left) {
        // sharded heads (psrt_kernels.h kQueues): global ticket g = t * kQueues + h
        while (qnext < (unsigned)kQueues) {
          const unsigned h = (blockIdx.x + qnext) % kQueues;
          uint64_t tk = 0;
          if (lane == 0) tk = atomicAdd(a.work_counter + kShardStride * h, 1ull);
          tk = __shfl(tk, 0);
          nb = (tk * kQueues + h) * kMatChunk;
          if (nb < total) {
            fresh = true;
            break;
          }
          ++qnext;
        }
      }
      if (!active) {
        uint64_t unit = ~0ull;
        if (rank < win_left) unit = win_base + rank;
        else if (fresh) unit = nb + (rank - win_left);
        if (unit < total) {
          su = (unsigned)unit;
          setup(su, rng, ox, oy, oz, dx, dy, dz, A, pq);
          PSRT_MAT_ABLATE_AT(SETUP);
          k = 0;
          np = 0;
          active = true;
        }
      }
      if (cnt > win_left) {
        if (fresh) {
          win_base = nb + (cnt - win_left);
          win_left = kMatChunk - (cnt - win_left);
        } else {
          win_left = 0;
          exhausted = true;
        }
      } else {
        win_base += cnt;
        win_left -= cnt;
      }
    }
    if (__ballot(active) == 0) break;

    // ---- world.hit(r, 0.001, inf) of this bounce (book ch. 9-10) ----
    bool fin = false, resolved = false, decided = false;
    double cr = 0.0, cg = 0.0, cb = 0.0;  // black: depth exhausted or absorbed
    if (active && !pending) {
      if (k >= a.max_depth) {
        fin = true;  // depth <= 0
      } else {
        ++rays;
        unsigned zg = 0;
        asm volatile("" : "+v"(zg));  // re-read the grid constants from LDS here
        const GridC& gc = *(const GridC*)((const char*)&s_gc + zg);
        __builtin_amdgcn_s_setprio(kMatHitPrio);
        uint4 rec = make_uint4(kCamOverflow, 0u, 0u, 0u);
        if (k == 0 && a.plist) rec = a.plist[pq];  // camera ray: its pixel's list
        decided = hit_quick_m<kBVH>(ntests, nroots, lgeo, a.n, bv, big_idx, gc, rec, ox, oy, oz,
                                    dx, dy, dz, A, pbt, pbi);
        PSRT_MAT_ABLATE_AT(HIT);
        __builtin_amdgcn_s_setprio(0);
        pending = !decided;
      }
    }
    if constexpr (kBVH) {
      const uint64_t pend = __ballot(pending);
      if (pend != 0 && ((unsigned)__popcll(pend) >= a.batch ||
                        __ballot(active && !pending && !fin) == 0)) {
        __builtin_amdgcn_s_setprio(kMatWalkPrio);
        if (pending) {
          PSRT_MAT_ABLATE_AT(WALK_SAVE);
          hit_walk_m(ntests, nboxes, nroots, bv, nodes, leaf_geo, leaf_idx, ox, oy, oz, dx, dy, dz,
                     A, pbt, pbi);
          PSRT_MAT_ABLATE_AT(WALK_RUN);
          pending = false;
          decided = true;
        }
        __builtin_amdgcn_s_setprio(0);
      }
    }
    if (decided) {
      if (pbi < 0) {
        // sky (main.cc:46-48), then attenuation * (...) innermost first
        const double y = (1.0 / __builtin_sqrt(A)) * dy;
        const double t = 0.5 * (y + 1.0);
        cr = (1.0 - t) * 1.0 + t * 0.5;
        cg = (1.0 - t) * 1.0 + t * 0.7;
        cb = (1.0 - t) * 1.0 + t * 1.0;
        for (int e = np - 1; e >= 0; --e) {
          double ar, ag, ab;
          mat_albedo(path[(size_t)e * ps], ar, ag, ab);
          cr = ar * cr;
          cg = ag * cg;
          cb = ab * cb;
        }
        fin = true;
      } else {
        resolved = true;
      }
    }

    // ---- scatter ----
    if (resolved) {
      const int bi = pbi;
      const HitRec h = hit_record_of(lgeo[bi], linv[bi], pbt, ox, oy, oz, dx, dy, dz);
      PSRT_MAT_ABLATE_AT(RECORD);
      const int kind = mat_kind(bi);
      double ndx = 0.0, ndy = 0.0, ndz = 0.0;
      bool ok = true;
      if (kind == RT_MAT_DIELECTRIC) {
        const double inv = 1.0 / __builtin_sqrt(A);
        const double ux = inv * dx, uy = inv * dy, uz = inv * dz;
        const double ir = mat_ir(bi);
        const double ratio = h.front ? (1.0 / ir) : ir;
        const double ct = __builtin_fmin(((-ux) * h.nx + (-uy) * h.ny) + (-uz) * h.nz, 1.0);
        const double st = __builtin_sqrt(1.0 - ct * ct);
        // cannot_refract || reflectance(...) > random_double(): the draw is
        // made only when refraction is possible
        const bool reflect = ratio * st > 1.0 || reflectance(ct, ratio) > random_double(rng);
        if (reflect) {  // reflect(v, n) = v - 2*dot(v,n)*n
          const double dn = (ux * h.nx + uy * h.ny) + uz * h.nz;
          ndx = ux - (2.0 * dn) * h.nx;
          ndy = uy - (2.0 * dn) * h.ny;
          ndz = uz - (2.0 * dn) * h.nz;
        } else {  // refract(uv, n, ratio), cos_theta = ct
          const double qx2 = ratio * (ux + ct * h.nx);
          const double qy2 = ratio * (uy + ct * h.ny);
          const double qz2 = ratio * (uz + ct * h.nz);
          const double par =
              -__builtin_sqrt(__builtin_fabs(1.0 - ((qx2 * qx2 + qy2 * qy2) + qz2 * qz2)));
          ndx = qx2 + par * h.nx;
          ndy = qy2 + par * h.ny;
          ndz = qz2 + par * h.nz;
        }
      } else {
        // random_in_unit_sphere() (vec3.h:83-95): trials of raw z, y, x draws
        // (g++'s order, vec3.h:78-81) until one lies in the ball; lambertian
        // and metal lanes share this one loop. (A look-ahead of trials generated
        // a loop iteration ahead, as psrt_trace keeps, was measured 11% slower
        // here: DESIGN.md §14.)
        // The acceptance test stays in FP64 here: psrt_trace's FP32
        // pre-decision (psrt_device.h in_unit_sphere_raw_f32) was 1.5% slower
        // in this divergent loop (its ballot runs per trial; r04,
        // profiles/r04_mat/ab.txt).
        PSRT_MAT_ABLATE_AT(TRIALS);
        uint32_t rz, ry, rx;
        for (;;) {
          raw32_x3(rng, rz, ry, rx, rng);
          if (in_unit_sphere_raw(rx, ry, rz)) break;
        }
        // random(-1, 1) of each draw, exact from the raw value (psrt_device.h)
        const double x = pm1_raw(rx), y = pm1_raw(ry), z = pm1_raw(rz);
        if (kind == RT_MAT_LAMBERTIAN) {
          // normal + random_unit_vector(); the normal if that is near zero
          const double inv = 1.0 / __builtin_sqrt((x * x + y * y) + z * z);
          ndx = h.nx + inv * x;
          ndy = h.ny + inv * y;
          ndz = h.nz + inv * z;
          if (__builtin_fabs(ndx) < 1e-8 && __builtin_fabs(ndy) < 1e-8 &&
              __builtin_fabs(ndz) < 1e-8)
            ndx = h.nx, ndy = h.ny, ndz = h.nz;
        } else {
          // metal: reflect(unit(d), n) + fuzz * random_in_unit_sphere();
          // absorbed unless outward
          const double inv = 1.0 / __builtin_sqrt(A);
          const double ux = inv * dx, uy = inv * dy, uz = inv * dz;
          const double dn = (ux * h.nx + uy * h.ny) + uz * h.nz;
          const double fz = mat_fuzz(bi);
          ndx = (ux - (2.0 * dn) * h.nx) + fz * x;
          ndy = (uy - (2.0 * dn) * h.ny) + fz * y;
          ndz = (uz - (2.0 * dn) * h.nz) + fz * z;
          ok = ((ndx * h.nx + ndy * h.ny) + ndz * h.nz) > 0.0;
        }
      }
      if (!ok) {
        fin = true;
      } else {
        if (kind != RT_MAT_DIELECTRIC) path[(size_t)np++ * ps] = bi;
        ox = h.px, oy = h.py, oz = h.pz;
        dx = ndx, dy = ndy, dz = ndz;
        A = (dx * dx + dy * dy) + dz * dz;
        ++k;
      }
    }
    if (fin) {
      double* const o = rgb + 3 * (size_t)su;
      o[0] = cr;
      o[1] = cg;
      o[2] = cb;
      active = false;
    }
  }
  // rays (== traced rays: no trapped-path shortcut here) -> this block's counter set
  unsigned long long* const ctr = a.ray_counter + kShardStride * (blockIdx.x % kQueues);
  for (int off = 32; off > 0; off >>= 1) rays += __shfl_xor(rays, off);
  if (lane == 0 && rays) {
    atomicAdd(ctr, rays);
    atomicAdd(ctr + 3, rays);
  }
  if constexpr (kCount) {
    unsigned long long t = ntests.v, b = nboxes.v, r = nroots.v;
    for (int off = 32; off > 0; off >>= 1)
      t += __shfl_xor(t, off), b += __shfl_xor(b, off), r += __shfl_xor(r, off);
    if (lane == 0) {
      atomicAdd(ctr + 1, t);
      atomicAdd(ctr + 2, b);
      atomicAdd(ctr + 5, r);
    }
  }
}

#define PSRT_MAT_INSTANTIATE1(B, L, C)                                                     \
  template __global__ void psrt_trace_mat<B, L, C>(const double4* __restrict__,             \
                                                   const double* __restrict__,              \
                                                   double* __restrict__, MatArgs, BvhView);
#define PSRT_MAT_INSTANTIATE(B, L) PSRT_MAT_INSTANTIATE1(B, L, false) PSRT_MAT_INSTANTIATE1(B, L, true)
PSRT_MAT_INSTANTIATE(false, false)
PSRT_MAT_INSTANTIATE(true, false)
PSRT_MAT_INSTANTIATE(true, true)
#undef PSRT_MAT_INSTANTIATE1
#undef PSRT_MAT_INSTANTIATE

// pixel_color += sample (main.cc:77-84) over colour records, in sample order;
// write_color (color.h:8-24) on the last chunk. One lane per pixel; block 0
// folds the trace launch's counter sets as psrt_reduce does.
__global__ __launch_bounds__(kReduceBlock) void psrt_reduce_rgb(ReduceArgs a) {
  if (blockIdx.x == 0 && a.fold_stats) {
    if (threadIdx.x < kStatWords) {
      unsigned long long v = a.first_chunk ? 0ull : a.totals[threadIdx.x];
      for (int h = 0; h < kQueues; ++h) {
        v += a.sets[kShardStride * h + threadIdx.x];
        a.sets[kShardStride * h + threadIdx.x] = 0ull;
      }
      a.totals[threadIdx.x] = v;
      if (a.host_stats) a.host_stats[threadIdx.x] = v;
    }
    if (threadIdx.x < kQueues) a.heads[kShardStride * threadIdx.x] = 0ull;
  }
  // One wave per 64 pixels. The 64 pixels' records are one contiguous run
  // ([pixel][s_count][3] doubles), so the wave stages tiles of kRgbTile
  // samples per pixel through LDS: 16-B loads spread over the lanes
  // (consecutive lanes, consecutive 16-B pieces of a pixel's tile), not one
  // 8-B load per lane per value at a pixel-run stride; then each lane adds its
  // pixel's samples in order (main.cc:77-84).
  constexpr unsigned kRgbTile = 8, kRow = kRgbTile * 3 + 1;  // doubles per LDS row (+1: banks)
  __shared__ double s_c[kReduceBlock * kRow];
  const unsigned lane = threadIdx.x;
  const unsigned q0 = blockIdx.x * kReduceBlock;
  const unsigned q = q0 + lane;
  const unsigned S = (unsigned)a.s_count;
  const unsigned np = min((unsigned)kReduceBlock, a.pixels > q0 ? a.pixels - q0 : 0u);
  double r = 0.0, g = 0.0, b = 0.0;
  if (!a.first_chunk && q < a.pixels) {
    r = a.accum[(size_t)q * 3 + 0];
    g = a.accum[(size_t)q * 3 + 1];
    b = a.accum[(size_t)q * 3 + 2];
  }
  const double* __restrict__ run = a.samp_t + (size_t)q0 * S * 3;
  for (unsigned s0 = 0; s0 < S; s0 += kRgbTile) {
    const unsigned T = min(kRgbTile, S - s0);
    const unsigned per = 3 * T;  // doubles of one pixel's tile
    __syncthreads();
    if (S % 2 == 0 && T % 2 == 0 && ((uintptr_t)run & 15u) == 0) {
      // 16-B pieces: pixel p's tile starts 16-B aligned (the run is, and S * 3
      // and s0 * 3 are even)
      const unsigned pieces = per / 2;
      for (unsigned e = lane; e < np * pieces; e += kReduceBlock) {
        const unsigned p = e / pieces, j = (e - p * pieces) * 2;
        const double2 v = *(const double2*)(run + (size_t)p * S * 3 + s0 * 3 + j);
        s_c[p * kRow + j] = v.x;
        s_c[p * kRow + j + 1] = v.y;
      }
    } else {
      for (unsigned e = lane; e < np * per; e += kReduceBlock) {
        const unsigned p = e / per, j = e - p * per;
        s_c[p * kRow + j] = run[(size_t)p * S * 3 + s0 * 3 + j];
      }
    }
    __syncthreads();
    if (q < a.pixels) {
      const double* c = s_c + lane * kRow;
      for (unsigned j = 0; j < T; ++j) {
        r += c[3 * j + 0];
        g += c[3 * j + 1];
        b += c[3 * j + 2];
      }
    }
  }
  if (q >= a.pixels) return;
  if (a.accum) {
    a.accum[(size_t)q * 3 + 0] = r;
    a.accum[(size_t)q * 3 + 1] = g;
    a.accum[(size_t)q * 3 + 2] = b;
  }
  if (a.rgb8) {
    const double inv = 1.0 / (double)a.spp_total;
    const double cc[3] = {r, g, b};
    for (int ch = 0; ch < 3; ++ch) {
      double x = __builtin_sqrt(cc[ch] * inv);
      x = (x < 0.0) ? 0.0 : x;      // std::max(x, 0.0)
      x = (0.999 < x) ? 0.999 : x;  // std::min(x, 0.999)
      a.rgb8[(size_t)q * 3 + ch] = (unsigned char)(int)(255.999 * x);
    }
  }
}

// ---- camera-ray candidate lists through the thin lens ----
//
// A camera ray of pixel (i, j) starts at x = o + offset, |x - o| <= rho (the
// lens radius; u, v are unit axes), and passes through a point y of the
// pixel's patch Q of the focus plane: y = (llc + s h) + t v with s in
// [i, i+1]/(W-1), t in [j, j+1]/(H-1) (main.cc:80-81). With the patch centre
// q_c, L = |q_c - o|, the axis a = (q_c - o)/L and r_Q = max |y - q_c| (at a
// corner: Q is a parallelogram), the ray's point x + u (y - x), u >= 0, lies
// within |1-u| rho + u r_Q <= rho + u (rho + r_Q) of o + u (q_c - o). So every
// ray of the pixel lies in the cone of apex o, axis a and half-angle
// asin((rho + r_Q)/L), dilated by rho; a sphere can return an accepted root
// only if its padded ball (r + pad, the BVH's root-error pad) dilated by rho
// meets that cone. The FP64 cone is widened (k by 2^-20 relative, the angle by
// 1e-9 rad, the ball by 2^-20), margins far above its own rounding. The tile
// and per-pixel passes follow psrt_camera_lists; rho = 0 is the pinhole.

namespace {

struct LensCone {
  double ax, ay, az, ca, sa;  // unit axis, cos / sin of the widened half-angle
  bool ok;
};

__device__ __forceinline__ void focus_point(const MatCamListArgs& a, double s, double t,
                                            double q[3]) {
#pragma unroll
  for (int k = 0; k < 3; ++k) q[k] = (a.llc[k] + s * a.hor[k]) + t * a.ver[k];
}

__device__ __forceinline__ LensCone lens_cone(const MatCamListArgs& a, double s0, double s1,
                                              double t0, double t1) {
  LensCone c;
  double qc[3];
  focus_point(a, 0.5 * (s0 + s1), 0.5 * (t0 + t1), qc);
  const double dx = qc[0] - a.org[0], dy = qc[1] - a.org[1], dz = qc[2] - a.org[2];
  const double L = __builtin_sqrt((dx * dx + dy * dy) + dz * dz);
  c.ax = dx / L, c.ay = dy / L, c.az = dz / L;
  double rq = 0.0;
  const double ss[2] = {s0, s1}, ts[2] = {t0, t1};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    double y[3];
    focus_point(a, ss[e & 1], ts[e >> 1], y);
    const double ex = y[0] - qc[0], ey = y[1] - qc[1], ez = y[2] - qc[2];
    rq = __builtin_fmax(rq, __builtin_sqrt((ex * ex + ey * ey) + ez * ez));
  }
  const double k = (a.lens_radius + rq) / L * (1.0 + 0x1p-20) + 1e-12;
  c.ca = __builtin_sqrt(__builtin_fmax(0.0, 1.0 - k * k)) - 1e-9;  // cos(asin k), widened
  c.sa = __builtin_sqrt(__builtin_fmax(0.0, 1.0 - c.ca * c.ca));
  c.ok = L > 0.0 && L < 1e300 && k < 0.99 && c.ca > 0.1;  // narrow, finite cone (else no lists)
  return c;
}

// Does the ball (centre s.xyz, radius sqrt(s.w) + pad + rho) meet the cone?
__device__ __forceinline__ bool lens_cone_meets(const LensCone& c, const MatCamListArgs& a,
                                                const double4 s) {
  const double cx = s.x - a.org[0], cy = s.y - a.org[1], cz = s.z - a.org[2];
  const double l2 = (cx * cx + cy * cy) + cz * cz;
  const double R = (__builtin_sqrt(s.w) + a.pad + a.lens_radius) * (1.0 + 0x1p-20);
  if (!(l2 > R * R * (1.0 + 0x1p-20))) return true;  // apex inside / near the ball (or NaN)
  const double l = __builtin_sqrt(l2);
  const double cb = ((c.ax * cx + c.ay * cy) + c.az * cz) / l;
  if (cb >= c.ca) return true;  // centre inside the cone
  const double sb = __builtin_sqrt(__builtin_fmax(0.0, 1.0 - cb * cb));
  // angle(axis, centre) - half-angle must be <= asin(R / l) (<= pi/2)
  const double cosd = cb * c.ca + sb * c.sa, sind = sb * c.ca - cb * c.sa;
  return cosd >= 0.0 && sind <= R / l;
}

}  // namespace

__global__ __launch_bounds__(64) void psrt_mat_camera_lists(MatCamListArgs a) {
  __shared__ int s_tile[kCamTileCap];
  const unsigned lane = __lane_id();
  const int x0 = blockIdx.x * kCamTile, r0 = blockIdx.y * kCamTile;
  const int x1 = min(x0 + kCamTile, a.width), r1 = min(r0 + kCamTile, a.rows);
  const int px = x0 + (int)(lane % kCamTile), rk = r0 + (int)(lane / kCamTile);
  const double iw = 1.0 / (double)(a.width - 1), ih = 1.0 / (double)(a.height - 1);
  // reference rows j = H-1-r fall as the shard row rk rises (main.cc:72)
  const int jhi = a.height - 1 - (a.row_offset + r0 * a.row_stride);
  const int jlo = a.height - 1 - (a.row_offset + (r1 - 1) * a.row_stride);
  // s, t bounds widened by a relative 2^-40 (the rounding of i + random_double()
  // and of the division)
  const double wid = 1.0 + 0x1p-40;
  const LensCone tc = lens_cone(a, x0 * iw / wid, x1 * iw * wid, jlo * ih / wid,
                                (jhi + 1) * ih * wid);
  int cnt = 0;
  bool over = !tc.ok;
  for (int base = 0; base < a.n_leaf && !over; base += 64) {
    const int k = base + (int)lane;
    const bool cand = k < a.n_leaf && lens_cone_meets(tc, a, a.leaf_geo[k]);
    const uint64_t m = __ballot(cand);
    const int pos = cnt + (int)lanes_below(m);
    if (cand && pos < kCamTileCap) s_tile[pos] = k;
    cnt += __popcll(m);
    if (cnt > kCamTileCap) over = true;
  }
  __syncthreads();
  if (px >= a.width || rk >= a.rows) return;
  const int j = a.height - 1 - (a.row_offset + rk * a.row_stride);
  unsigned w[4] = {kCamOverflow, 0u, 0u, 0u};
  if (!over) {
    const LensCone pc = lens_cone(a, px * iw / wid, (px + 1) * iw * wid, j * ih / wid,
                                  (j + 1) * ih * wid);
    unsigned n = 0;
    bool full = !pc.ok;
    for (int e = 0; e < cnt && !full; ++e) {
      const int k = s_tile[e];
      if (!lens_cone_meets(pc, a, a.leaf_geo[k])) continue;
      if (n == (unsigned)kCamPixelCap) {
        full = true;
        break;
      }
      ++n;  // slot n of 8 uint16 (slot 0 = count)
      w[n >> 1] |= (unsigned)a.leaf_idx[k] << ((n & 1) * 16);
    }
    if (!full) w[0] = (w[0] & 0xFFFF0000u) | n;
  }
  a.plist[(size_t)rk * a.width + px] = make_uint4(w[0], w[1], w[2], w[3]);
}

}  // namespace psrt
