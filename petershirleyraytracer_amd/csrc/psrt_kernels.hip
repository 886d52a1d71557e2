// psrt_kernels.hip — gfx950 kernels of the path-tracing hot path.
//
//   psrt_trace    the megakernel: persistent lanes, one camera sample per
//                 work unit, the ray_color recursion (main.cc:34-49) as a
//                 bounce loop, hittable_list::hit / sphere::hit
//                 (hittable_list.cc:3-20, sphere.cc:3-40) as a sweep over the
//                 flattened sphere list, diffuse scatter (vec3.h:83-109).
//                 A lane whose path ends stores that sample's colour and is
//                 refilled from the wave's work window in the same iteration
//                 (ballot + mbcnt), so every iteration every lane carries a
//                 live ray until the queue drains.
//   psrt_reduce   pixel_color += sample (main.cc:77-84) in sample order,
//                 then write_color (color.h:8-24) on the last chunk.
//
// Data layout in HBM:
//   geo[n]      double4 {cx, cy, cz, r*r}   sphere.cc:11 radius*radius
//   inv_r[n]    double  1.0/r              vec3.h:151-154 (1/t)*v
//   samples     double[P][s_count] t, uint16[P][s_count] k: sample s of pixel q at
//               unit q*s_count + s (sample_colour)
//                                          (sample_colour)
//   accum       double[P][3]               P = rows_owned * W, reference order
//   rgb8        uint8 [P][3]
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "psrt_device.h"
#include "psrt_kernels.h"
#include "psrt_geom.h"

namespace psrt {

// Wave issue priorities (s_setprio; DESIGN.md §4 "Issue priorities"): a wave
// raises its priority during the latency-bound sections (the batched BVH
// walk, hit_quick) and, once the work queue is empty, keeps a raised base
// priority for the launch tail (TraceArgs::tail_prio).
constexpr int kWalkPrio = 3;
constexpr int kHitPrio = 2;
constexpr int kTailPrio = 1;
// Minimum waves per SIMD asked of the register allocator (80 VGPRs).
constexpr int kTraceWaves = 6;
// Loop schedule (tuned; re-swept under multi-frame launches in r03,
// profiles/r03_knobs): compile-time constants, so they take no SGPRs in the
// loop (held as kernel arguments they pushed SGPRs into VGPR-lane spills).
#ifndef PSRT_REFILL_MIN
#define PSRT_REFILL_MIN 16
#endif
#ifndef PSRT_WALK_BATCH
#define PSRT_WALK_BATCH 24
#endif
constexpr unsigned kRefillMin = PSRT_REFILL_MIN;  // idle lanes that trigger the finish + refill block
constexpr unsigned kWalkBatch = PSRT_WALK_BATCH;  // parked lanes that trigger a batched BVH pass
#ifndef PSRT_WALK_TAIL
#define PSRT_WALK_TAIL 6  // r04 re-sweep (profiles/r04_knobs2): 2 / 4 / 6 / 8
#endif
constexpr unsigned kWalkTail = PSRT_WALK_TAIL;  // a BVH pass stops once this few lanes still walk
#ifndef PSRT_RNG_FILL
#define PSRT_RNG_FILL 2
#endif
#ifndef PSRT_RNG_EXTRA
#define PSRT_RNG_EXTRA 1
#endif
constexpr int kRngFill = PSRT_RNG_FILL;    // look-ahead trials per lane per iteration (min)
constexpr int kRngExtra = PSRT_RNG_EXTRA;  // extra trials while a scattering lane has none queued

__device__ __forceinline__ unsigned lane_id() { return __lane_id(); }

// Section ablation for the census: measurement builds only
// (PSRT_ABLATE = section id, psrt_ablate.h); in the product build every
// PSRT_ABLATE_AT hook is empty.
#ifndef PSRT_ABLATE
#define PSRT_ABLATE 0
#endif
#if PSRT_ABLATE
#include "psrt_ablate.h"
#else
#define PSRT_ABLATE_AT(site)
#endif

// Diagnostic build only (kStamps): wave-level cycle accounting per kernel
// section, one s_memtime per boundary (cdna_hip_programming.md §7 stamps).
// Read its SHARES, never its run time.
enum Section {
  kSecRefill = 0, kSecHit, kSecScatter, kSecFillShade, kSecTraverse,
  kSecQHint, kSecQBig, kSecQGrid, kSecCount  // hit_quick sub-sections (share of kSecHit)
};

// Lane utilisation probes (diagnostic build): per probe, wave executions and
// active lanes, counted by the first active lane.
enum Util { kURefill = 0, kUStore, kUHit, kUHint, kUNb, kUCam, kUGrid, kUWalk, kUTrial,
            kUScatter,
            // hit_quick outcomes (lanes per wave execution, counted where decided)
            kUHintHit, kUHintTiny, kUGridCell, kUGridOut, kUGridNoneFin, kUGridNoneInf,
            kUFarMiss, kUPark, kUListTrip,
            // walk outcomes: {rays, summed box tests} by result (BVH sphere / big / none)
            // and by whether the ray parked with a finite bound
            kUWBvh, kUWBig, kUWMiss, kUWFin, kUWInf, kUCount };

__device__ __forceinline__ bool first_active_lane();

template <bool kOn>
struct SectionClock {
  uint64_t t = 0, acc[kSecCount] = {0, 0, 0, 0, 0, 0, 0, 0};
  // utilisation probes: {wave executions, active lanes} per probe, in the
  // workgroup's LDS (LDS atomics by the first active lane); flushed at exit
  unsigned* ucnt = nullptr;
  __device__ __forceinline__ void util(int u) {
#ifdef PSRT_STAMPS_NO_UTIL  // section clocks only: no LDS atomics inside the sections
    if constexpr (false) {
#else
    if constexpr (kOn) {
#endif
      const uint64_t m = __ballot(1);
      if (first_active_lane()) {
        atomicAdd(ucnt + 2 * u, 1u);
        atomicAdd(ucnt + 2 * u + 1, (unsigned)__popcll(m));
      }
    }
  }
  // diagnostic: per lane, {lanes, sum of v} into probe u (LDS atomics)
  __device__ __forceinline__ void add(int u, unsigned v) {
    if constexpr (kOn) {
      atomicAdd(ucnt + 2 * u, 1u);
      atomicAdd(ucnt + 2 * u + 1, v);
    }
  }
  __device__ __forceinline__ void start() {
    if constexpr (kOn) t = now();
  }
  __device__ __forceinline__ void mark(int sec) {
    if constexpr (kOn) {
      const uint64_t n = now();
      acc[sec] += n - t;
      t = n;
    }
  }
  static __device__ __forceinline__ uint64_t now() {
    uint64_t v;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return v;
  }
};

constexpr unsigned kDrainEvery = 64;  // workgroups per drain-flag writer (TraceArgs::drain_flag)

struct RefillConst {
  // guided work queue phases (TraceArgs::ph_*), read when a wave takes a ticket
  uint64_t ph_first[kQueuePhases + 1];
  uint64_t ph_base[kQueuePhases];
  unsigned ph_size[kQueuePhases];
  double cam[12];  // origin, lower_left, horizontal, vertical
  double wm1, hm1;  // (double)(W - 1), (double)(H - 1)   main.cc:80-81
  double rwm1, rhm1;  // RN(1 / wm1), RN(1 / hm1), or 0 when the divisor is 0 (div_by)
  uint64_t seedmix[kMaxFrames];  // splitmix64(seed of frame f) (TraceArgs::frames)
  FastDiv div_s, div_w, div_p;
  int hm1_i, row_offset, row_stride, s_begin, frames;
  unsigned long long* drain_flag;  // TraceArgs::drain_flag / drain_epoch
  unsigned long long drain_epoch;
};

__device__ __forceinline__ unsigned fast_div(unsigned n, const FastDiv& f) {
  const unsigned t = __umulhi(f.m, n);
  return (t + ((n - t) >> f.sh1)) >> f.sh2;
}

// x / d, correctly rounded, for x >= 0 and d >= 1 from y = RN(1/d) (the
// camera ray's u and v, main.cc:80-81): q0 = RN(x y) is within 1.5 ulp of
// x/d; one correction q1 = RN(q0 + RN(x - d q0) y) brings it within
// 0.5 + 2^-50 ulp; with q1 within 1 ulp, r1 = x - d q1 is exact and
// RN(q1 + r1 y) = RN(x/d) (Markstein's theorem). No intermediate under- or
// overflows for these operands (x < 2^31, d < 2^31); x = 0 gives +0. Five
// FP64 ops instead of the division's ten and a v_rcp_f64.
__device__ __forceinline__ double div_by(double x, double d, double y) {
  double q = x * y;
  double r = __builtin_fma(-q, d, x);
  q = __builtin_fma(r, y, q);
  r = __builtin_fma(-q, d, x);
  return __builtin_fma(r, y, q);
}

__device__ __forceinline__ unsigned mbcnt64(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32),
                                   __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
}

// 0.5^k * x as the reference's k nested `0.5 * ray_color(...)` (main.cc:43).
// x >= 0.5 here, so ldexp is exact (= the k products) while 2^-k*x stays
// normal; past that the products are taken one by one as the reference does.
__device__ __forceinline__ double half_pow(double x, int k) {
  if (k <= 1000) return __builtin_ldexp(x, -k);
  for (int m = 0; m < k; ++m) x = 0.5 * x;
  return x;
}

// A sample's colour (main.cc:43-48): black, or the sky at t = 0.5 (y + 1)
// (y: the last ray's unit direction) times 0.5^k, k = hits on the path. The
// trace stores (t, k) and psrt_reduce forms the colour, with the same FP64
// operations in the same order. k is stored capped at kSampleKCap: from
// ~1076 halvings on, x <= 1 is +0 (and NaN stays NaN), so the cap changes no bit.
__device__ __forceinline__ void sample_colour(double tt, unsigned short kk, double& r, double& g,
                                              double& b) {
  r = g = b = 0.0;
  if (kk != kSampleBlack) {
    const double w = 1.0 - tt;
    r = half_pow(w + tt * 0.5, kk);
    g = half_pow(w + tt * 0.7, kk);
    b = half_pow(w + tt * 1.0, kk);
  }
}



// Root selection of sphere.cc:24-31 over [0, tmax], bit for bit, with one
// division where the reference may take two: the near root t1 = n1/A
// (n1 = -hb - sq) is certainly < 0, and not -0, when n1 < -A*2^-900 (also
// when A*2^-900 underflows: then |n1/A| >= 2^-1074/A > 2^-952); the far root
// then decides, as in the reference. If t1 > tmax the far root is rejected
// too: -hb + sq >= -hb - sq after rounding and division by A > 0 is
// monotone, so t2 >= t1. A second division runs only for t1 in (-2^-900, 0),
// behind a wave-uniform branch: left to itself the compiler if-converts it and
// every test pays both divisions (~13 VALU instructions and a v_rcp_f64 each).
// NaN roots pass, as in the reference. Returns whether the root t is taken.
__device__ __forceinline__ bool root_select(double hb, double sq, double A, double tmax,
                                            double& t) {
  const double n1 = -hb - sq;
  const bool far = n1 < -(A * 0x1p-900);
  t = (far ? -hb + sq : n1) / A;
  const bool again = !far && t < 0.0;
  if (__builtin_expect(__ballot(again) != 0, 0)) {
    if (again) t = (-hb + sq) / A;
  }
  return !(t < 0.0 || t > tmax);
}

// Sphere sweep of hittable_list::hit(r, tmin, tmax, rec) (hittable_list.cc:3-20
// over sphere.cc:3-33). Only the winner's record is formed afterwards
// (hit_record_of): every earlier accepted record is overwritten in the
// reference, so the result is the same. Ties go to the later index
// (sphere.cc:26 accepts t == tmax). NaN follows the reference: a NaN
// discriminant is not "< 0" and a NaN root passes both range tests.
// With kFix (the small-scene trace path), it also decides the trapped-path
// test of §9 on the way: C == 0 on the hint sphere, and every other sphere
// clear of the origin (the direction-free part of test_sphere's pre-reject).
template <bool kFix = false>
__device__ __forceinline__ int sweep_linear(const double4* __restrict__ geo, int n, double ox,
                                            double oy, double oz, double dx, double dy, double dz,
                                            double A, double tmin, double tmax, double& best_t,
                                            int hint = -1, bool* trapped = nullptr) {
  int best_i = -1;
  double closest = tmax;
  bool fix = false, clear = true;
  for (int i = 0; i < n; ++i) {
    const double4 s = geo[i];
    const double ax = ox - s.x, ay = oy - s.y, az = oz - s.z;
    const double hb = (dx * ax + dy * ay) + dz * az;
    const double c = ((ax * ax + ay * ay) + az * az) - s.w;
    if constexpr (kFix) {
      if (i == hint) {
        fix = c == 0.0 && s.w >= 0x1p-700 && s.w <= 0x1p700;
      } else {
        const double k2 = 2.0 * (c + 2.0 * s.w);
        clear = clear && c > 0.0 && c * c >= 0x1p-34 * (c + s.w) * k2;
      }
    }
    const double disc = hb * hb - A * c;
    if (!(disc < 0.0)) {
      const double sq = sqrt_f64(disc);
      double t;
      bool ok = true;
      if constexpr (kFix) {  // the trace path: tmin == 0
        ok = root_select(hb, sq, A, closest, t);
      } else {
        t = (-hb - sq) / A;
        if (t < tmin || t > closest) {
          t = (-hb + sq) / A;
          if (t < tmin || t > closest) ok = false;
        }
      }
      if (ok) {
        closest = t;
        best_i = i;
      }
    }
  }
  best_t = closest;
  if constexpr (kFix) *trapped = fix && clear && best_i == hint;
  return best_i;
}


// ---- exact culling ------------------------------------------
//
// The reference's list scan returns the lexicographic minimum of (tau_j, -j)
// over spheres with a root tau_j in [0, closest] (tau_j: near root if >= 0,
// else far root if >= 0 — independent of closest, sphere.cc:24-31). So any
// visiting order that evaluates every sphere whose root could land in
// [0, closest], with the same FP64 test, returns the same record. The BVH
// (psrt_bvh.h) visits a superset: its FP32 boxes are padded past the FP32
// slab error and the FP64 root error; rays it cannot bound (non-finite, A
// not in (0, 1e200), |o|inf > 8 r_check) take the linear sweep; origins
// between r_check and 8 r_check test the padded root box in FP64 first.

// sphere.cc:6-31 for one sphere, then the (t, index) rule of the list scan,
// after an exact pre-reject in FP32 (Pre32; r04, replacing r01-r03's FP64
// one). When the origin lies outside the sphere by D = |amc| - |r|, every
// root has t |d| >= D; the computed roots are within ~2^-25 |amc| of that
// (worst case: tangency, where the discriminant's rounding error is ~2^-52
// HALF_B^2). With o, c and A in range (below), let a = fl(fl(o) - fl(c)) per
// axis, L = fl(ax^2 + ay^2 + az^2) (two FMAs) and T = fl(fl(bt) sk +
// fl(mo + R)), where sk >= sqrt(A) (1 + 2^-17), mo >= 2^-18 |o|inf and
// R >= |r| + 2^-18 (|c|inf + |r|) + 2^-60 (host, rounded up; the floor keeps
// T^2 >= 2^-120 a normal float). Rounding
// analysis (u = 2^-24): |a - amc| <= 3.5u (|o|inf + |c|inf), L <= |a|^2
// (1 + 3.01u), fl(T T) >= T^2 (1 - u), so L > fl(T T) gives
// D > bt sqrt(A) (1 + 2^-18.1) + 2^-18.1 (|o|inf + |c|inf + |r|) >= bt sqrt(A)
// + 2^-20 |amc|: the computed roots exceed bt and the reference rejects them
// too. Out of range (|o|inf > 2^40, A outside [2^-100, 2^100], |c| or r
// beyond 2^40, bt = inf or beyond FP32) T, or T^2, is +inf or NaN and nothing
// is rejected. 10 VALU instructions, mostly FP32, where the FP64 form took
// ~20 FP64 ones (4 cycles each); its margin (2^-18 relative) rejects at the
// distances the FP64 one did (D >= 2^-17 |amc|). C3 psrt_trace 12.08 ->
// 11.80 ms (profiles/r04_pre32/ab.txt); tests/host/pre32_check.c checks it
// against the reference test on 8.2 M adversarial cases, at scene scales
// from 1 down to 2^-90.
// Returns false when the pre-reject decided the sphere, true when the full
// test ran. *c_out (if given) receives C = amc.amc - r^2 as sphere.cc:11 forms it.
struct Pre32 {
  float ox, oy, oz;  // fl(o)
  float sk;          // sqrt(fl(A)) (1 + 2^-16), or +inf: no pre-reject
  float mo;          // 2^-18 |o|inf (1 + 2^-20)
};

__device__ __forceinline__ Pre32 pre32_of(double ox, double oy, double oz, double A, double am) {
  Pre32 p;
  p.ox = (float)ox, p.oy = (float)oy, p.oz = (float)oz;
  const bool ok = am <= 0x1p40 && A >= 0x1p-100 && A <= 0x1p100;
  p.sk = ok ? __builtin_amdgcn_sqrtf((float)A) * (1.0f + 0x1p-16f) : __builtin_inff();
  p.mo = (float)am * (0x1p-18f * (1.0f + 0x1p-20f));
  return p;
}

template <bool kPre = true>
__device__ __forceinline__ bool test_sphere(const double4 s, int idx, double ox, double oy,
                                            double oz, double dx, double dy, double dz,
                                            double A, double& best_t, int& best_i,
                                            const float4 s32, const Pre32& pr,
                                            double* c_out = nullptr) {
  if (kPre) {
    const float ax = pr.ox - s32.x, ay = pr.oy - s32.y, az = pr.oz - s32.z;
    const float L = __builtin_fmaf(ax, ax, __builtin_fmaf(ay, ay, az * az));
    const float T = __builtin_fmaf((float)best_t, pr.sk, pr.mo + s32.w);
    if (L > T * T) return false;
  }
  const double ax = ox - s.x, ay = oy - s.y, az = oz - s.z;
  const double c = ((ax * ax + ay * ay) + az * az) - s.w;
  if (c_out) *c_out = c;
  const double hb = (dx * ax + dy * ay) + dz * az;
  const double disc = hb * hb - A * c;
  if (disc < 0.0) return true;
  const double sq = sqrt_f64(disc);
  double t;
  if (!root_select(hb, sq, A, best_t, t)) return true;
  if (t < best_t || idx > best_i) {  // equal t: the later index wins
    best_t = t;
    best_i = idx;
  }
  return true;
}



// A per-lane counter that counts nothing: the sphere / box test counters of
// psrt_trace<..., kCount = false>, the default kernel (RT_FLAG_CULL_STATS
// selects the counting one). Two fewer live VGPRs in the trace loop take its
// spills from 9 to 1 (-0.1 ms per C3 launch, r02).
struct NullCount {
  __device__ NullCount() = default;
  __device__ NullCount(unsigned) {}
  __device__ NullCount& operator+=(unsigned) { return *this; }
  __device__ NullCount& operator++() { return *this; }
  __device__ operator unsigned() const { return 0u; }
};
// What the counting variant tallies, by the kind of test that actually ran
// (bench.py weights each kind by its measured issue cost):
//   fp64   sphere tests run in full in FP64 (sphere.cc:6-31; the hint test,
//          big / listed / leaf spheres past the pre-reject, the linear sweep)
//   pre    sphere candidates decided by the FP32 pre-reject (Pre32) alone
//   boxes  FP32 slab tests evaluated in the BVH walk (node + 1's test only
//          when it ran)
//   root   FP64 root-box tests (far origins, hit_quick)
// Candidates skipped because they are the hint sphere count as nothing.
template <bool kCount>
struct CullStatsT {
  std::conditional_t<kCount, unsigned, NullCount> boxes, fp64, pre, root;
  // diagnostic build only: wave-level loop trips (counted by the first
  // active lane) vs lane-level work, to measure traversal divergence
  unsigned wave_trips = 0, wave_leaf_trips = 0, trav_rays = 0, leaf_visits = 0;
};
using CullStats = CullStatsT<true>;

__device__ __forceinline__ bool first_active_lane() {
  return __lane_id() == (unsigned)__builtin_ctzll(__ballot(1));
}

// Per-sphere data as the trace loop reads it: one LdsSphere record per sphere
// in LDS (kLds; psrt_kernels.h), else the separate global arrays.
template <bool kRec>
struct SphereView;
template <>
struct SphereView<true> {
  const LdsSphere* __restrict__ s;
  __device__ double4 geo(int i) const { return s[i].geo; }
  __device__ float4 g32(int i) const { return s[i].g32; }
  __device__ uint2 nb(int i) const { return s[i].nb; }
  __device__ double inv(int i) const { return s[i].inv; }
};
template <>
struct SphereView<false> {
  const double4* __restrict__ g;
  const float4* __restrict__ f;
  const uint2* __restrict__ b;
  const double* __restrict__ v;
  __device__ double4 geo(int i) const { return g[i]; }
  __device__ float4 g32(int i) const { return f[i]; }
  __device__ uint2 nb(int i) const { return b[i]; }
  __device__ double inv(int i) const { return v[i]; }
};

// Cheap part of hittable_list::hit with culling: the previous-hit sphere
// first, the big spheres, then the point-location grid. Returns true when the
// closest hit is decided (bt, bi); false when the BVH must be walked (the
// ray's bt, bi so far stay valid and hit_traverse continues from them).
//
// Trapped-path termination. Let the ray start at o on sphere j
// (the previous hit, `hint`) with C_j(o) = ((ax*ax + ay*ay) + az*az) - r*r
// computed as exactly 0. Then for EVERY direction d: A*C = +0, disc = fl(hb*hb),
// sqrt(fl(hb*hb)) = |hb| (binary64, no under/overflow), so sphere j's accepted
// root is t = +-0 and p = o + t*d equals o in value: the path never leaves o.
// If, besides, every other candidate sphere was decided without the full test
// (pre-rejected: origin outside, clear of the surface; or outside the grid
// cell / grid), each of those has no root <= 0 in any direction, so every
// later world.hit returns sphere j at t = +-0 again, whatever the draws. The
// path then hits until depth runs out: main.cc:36-37 returns black. The
// guards keep hb far from under/overflow for every reachable direction
// d = ((p + n) + rv) - p (n = +-(o - c)/r, rv in n's hemisphere, so
// |hb| >= r/2): 2^-700 <= r^2 <= 2^700 and |o|_inf <= 2^40.
template <class Clock, class CS, class SV>
__device__ __forceinline__ bool hit_quick(const double4* __restrict__ geo,
                                          const SV& sv, int n,
                                          const BvhView& bv, int hint, double ox, double oy,
                                          double oz, double dx, double dy, double dz, double A,
                                          double& bt, int& bi, CS& cs, Clock& clk,
                                          bool& trapped, unsigned q,
                                          const GridC& gc, const int* __restrict__ lbig,
                                          float& t0f) {
  bt = __builtin_inf();
  bi = -1;
  trapped = false;
  t0f = 0.0f;
  const bool finite = (A > 0.0) && (A < 1e200);
  const double am = __builtin_fmax(__builtin_fabs(ox),
                                   __builtin_fmax(__builtin_fabs(oy), __builtin_fabs(oz)));
  // Unbounded arithmetic, or an origin so far out (|o|inf > 8 r_check = 2^9 S)
  // that the reference's own roots may err by more than the BVH pad: a root's
  // point is good to ~1.5 x 2^-25 |o - c| near tangency, <= 2^-14.6 S (a third
  // of the pad) for |o - c| <= 2^9.8 S. The reference scan,
  // verbatim (NaN and infinities fail the test too).
  if (!finite || !(am * 0.125 <= gc.r_check)) {
    cs.fp64 += n;
    bi = sweep_linear(geo, n, ox, oy, oz, dx, dy, dz, A, 0.0, __builtin_inf(), bt);
    return true;
  }
  const Pre32 pr = pre32_of(ox, oy, oz, A, am);
  bool fix = false, full = false, nb = false;
  // The candidate list as an inline record {count | i0 << 16, i1 | i2 << 16,
  // ...} (uint16 slots, count kListOverflow = none): a camera ray's pixel list
  // (psrt_camera_lists), loaded early; the hint sphere's neighbour record or
  // the grid list's replace it below.
  uint4 rec = make_uint4(kCamOverflow, 0u, 0u, 0u);
  if (hint < 0 && gc.plist) rec = gc.plist[q];  // from LDS (GridC), not a spilled SGPR pair
  if (hint >= 0) {
    clk.util(kUHint);
    const double4 sh = sv.geo(hint);
    double ch;
    // the ray's first test: bt = +inf, so no pre-reject
    test_sphere<false>(sh, hint, ox, oy, oz, dx, dy, dz, A, bt, bi, float4{}, pr, &ch);
    PSRT_ABLATE_AT(HINT);
    fix = bv.fixpoint && ch == 0.0 && sh.w >= 0x1p-700 && sh.w <= 0x1p700 && am <= 0x1p40;
    ++cs.fp64;
    if (bi == hint) {
      clk.util(kUHintHit);
      if (bt < 1e-6) clk.util(kUHintTiny);
    }
    // Neighbour path: the hint sphere j was hit at bt and o
    // lies within pad/2 of its surface, so the segment [o, o + bt d] (both
    // ends in the ball of radius r_j + pad/2; the far end is a root of j, good
    // to ~2^-19 S) stays in that ball. A sphere with an accepted root t <= bt
    // has its hit point there and within the root error of its own surface,
    // so its centre lies within r_j + r_k + pad of c_j: it is j's neighbour.
    if (bi == hint && am <= gc.r_check && gc.nb_c2 >= 0.0 &&
        (ch <= 0.0 || ch * ch <= gc.nb_c2 * sh.w)) {
      const uint2 nr = sv.nb(hint);
      nb = (nr.x & 0xFFFFu) != kCamOverflow;
      if (nb) rec = make_uint4(nr.x, nr.y, 0u, 0u);
    }
  }
  clk.mark(kSecQHint);
  PSRT_ABLATE_AT(BIG);
  // the big spheres from the scene copy in LDS (kLds; the global arrays
  // otherwise): their indices, spheres and FP32 spheres
  for (int b = 0; b < bv.n_big; ++b) {
    const int idx = lbig[b];
    if (idx != hint) {
      const bool ran = test_sphere(sv.geo(idx), idx, ox, oy, oz, dx, dy, dz, A, bt, bi, sv.g32(idx), pr);
      full |= ran;
      cs.fp64 += ran;
      cs.pre += !ran;
    }
  }
  clk.mark(kSecQBig);
  // The candidate list of this ray, one of:
  //   neighbour list of the hint sphere (nb path), the pixel's camera list,
  //   or the grid cell holding [o, o + bt d];
  // all three are records of the same form, walked by ONE loop below, so a
  // wave whose lanes took different paths runs max(count) sphere tests
  // instead of their sum, and no trip loads anything but the sphere.
  bool listed = true;
  if (nb) {
    clk.util(kUNb);
  } else if ((rec.x & 0xFFFFu) != kCamOverflow) {
    // every BVH sphere a ray of this pixel can hit is listed
    clk.util(kUCam);
  } else {
    clk.util(kUGrid);
    // FP32 query, exact while its error (~4 ulp of the segment's coordinates)
    // stays below pad + margin = 1.25 pad (a hit point lies >= pad inside its
    // sphere's padded box): coordinates up to ~630 S; admitted up to 256 S
    // (|o| <= 4 r_check, bt |d| <= 4 r_check), else the walk / root-box test
    const double rg = 4.0 * gc.r_check;
    const int cell = (am <= rg && (bt * bt) * A <= rg * rg)
                         ? grid_locate(gc, ox, oy, oz, dx, dy, dz, bt) : kGridNone;
    listed = cell != kGridNone;
    if (cell >= 0) clk.util(kUGridCell);
    else if (cell == kGridOutside) clk.util(kUGridOut);
    else if (bt < 1e30) clk.util(kUGridNoneFin);
    else clk.util(kUGridNoneInf);
    if (cell >= 0) {
      rec = bv.cell_rec[cell];
      // a list too long for a record: the walk decides (exact either way)
      if ((rec.x & 0xFFFFu) == kCamOverflow) listed = false;
    } else {
      rec.x = 0u;
    }
  }
  const int cnt = listed ? (int)(rec.x & 0xFFFFu) : 0;
  uint64_t lo = rec.x | (uint64_t)rec.y << 32, hi = rec.z | (uint64_t)rec.w << 32;
  PSRT_ABLATE_AT(LIST);
  for (int e = 0; e < cnt; ++e) {
    clk.util(kUListTrip);
    lo = (lo >> 16) | (hi << 48);
    hi >>= 16;
    const int idx = (int)(lo & 0xFFFFu);
    if (idx == hint) continue;
    const bool ran = test_sphere(sv.geo(idx), idx, ox, oy, oz, dx, dy, dz, A, bt, bi, sv.g32(idx), pr);
    full |= ran;
    cs.fp64 += ran;
    cs.pre += !ran;
  }
  clk.mark(kSecQGrid);
  if (listed) {
    trapped = fix && !full && bi == hint;
    return true;
  }
  if (!(am <= gc.r_check)) {
    // Far origin (e.g. inside the r=1000 ground): test [0, bt] against the
    // padded root box in FP64 (error ~1e-13 relative, far inside the pad). A
    // miss proves no BVH sphere can have a root in [0, bt]; a hit parks the
    // ray for the batched walk, which re-bases it at the box entry (hit_traverse).
    ++cs.root;
    const double e = root_box_entry(bv, ox, oy, oz, dx, dy, dz, bt);
    if (e < 0.0) {
      clk.util(kUFarMiss);
      return true;
    }
    // The walk re-bases the ray here (hit_traverse). Any nearby point of the
    // ray serves: with |o|inf <= 2^9 S (the 8 r_check guard above) the float rounding of
    // e moves it by <= 2^-24 e |d| < 2^-14 S along the ray, and the re-based
    // origin stays in the range the slab test's error bound covers
    // (psrt_bvh.cpp; ADVICE r04 asked about origins beyond that range: they
    // take the linear scan).
    t0f = (float)e;
  }
  clk.util(kUPark);
  return false;
}


// The BVH walk (stackless, skip links) for a bounded ray, continuing from the
// (bt, bi) hit_quick left.
template <bool kDiag, bool kLdsLeaves, class CS, class SV>
__device__ __forceinline__ void hit_traverse(const BvhView& bv, const float4* __restrict__ nodes,
                                             const int* __restrict__ leaf_idx, const SV& sv,
                                             int hint,
                                             double ox, double oy, double oz, double dx, double dy,
                                             double dz, double A, double& bt, int& bi,
                                             CS& cs, int& node, unsigned tail, double t0) {
  // Far origins are re-based at their root-box entry o' = o + t0 d (FP64), so
  // the FP32 slab test sees |o'| <= the scene scale and its error bound holds;
  // box intervals are then tested over [-t0, bt - t0]. The exact sphere tests
  // in the leaves keep the original o.
  // t0: the entry hit_quick found (0 for near origins); a resumed walk keeps
  // it (a smaller bt only shortens [-t0, bt - t0])
  const double am = __builtin_fmax(__builtin_fabs(ox),
                                   __builtin_fmax(__builtin_fabs(oy), __builtin_fabs(oz)));
  const float fox = (float)(ox + t0 * dx), foy = (float)(oy + t0 * dy), foz = (float)(oz + t0 * dz);
  const float ix = safe_inv((float)dx), iy = safe_inv((float)dy), iz = safe_inv((float)dz);
  const float oix = fox * ix, oiy = foy * iy, oiz = foz * iz;
  const float tlo = -(float)t0 * 1.00000048f;  // <= -t0: the ray's t >= 0
  float tmax = tmax_up(bt - t0);
  if constexpr (kDiag) cs.trav_rays += node == bv.walk0;
  // Two nodes per trip: in DFS skip-link order an interior hit always
  // continues at node+1, so node+1 is loaded alongside node and, when node is
  // an interior hit, box-tested in the same trip; the trip then advances two
  // levels. Node n_nodes is a padding node (psrt_bvh.cpp), so node+1 is
  // always readable.
  //
  // While-while (Aila & Laine 2009): a lane that reaches a leaf stops and
  // holds it while the other lanes keep walking; the held leaves are then
  // tested together, so one pass of FP64 sphere tests serves every lane
  // that has a leaf instead of one pass per trip in which any lane has one.
  // A lane holding a leaf does not walk on, so its tmax is never stale.
  int leaf = -1;
  for (;;) {
    // tail cut: once no more than `tail` lanes still walk, they stop and keep
    // their node; they resume in the next pass with the newly parked rays
    const uint64_t walking = __ballot(node < bv.n_nodes);
    if (walking == 0 || (tail && (unsigned)__popcll(walking) <= tail)) break;
    while (node < bv.n_nodes && leaf < 0) {
      if constexpr (kDiag) {
        if (first_active_lane()) ++cs.wave_trips;
      }
      const float4 a0 = nodes[2 * node], a1 = nodes[2 * node + 1];
      const float4 b0 = nodes[2 * node + 2], b1 = nodes[2 * node + 3];
      // slab distances; FP32 FMA is fine here: the test only needs to be
      // conservative, and the box padding covers its rounding (psrt_bvh.cpp).
      // node+1's test runs only where node is an interior hit: the walk is
      // VALU-issue bound, so skipping it beats overlapping it (measured).
      const bool hit_a = slab_hit(a0, a1, ix, iy, iz, oix, oiy, oiz, tlo, tmax);
      const int leaf_a = __float_as_int(a1.w), leaf_b = __float_as_int(b1.w);
      int next;
      if (!hit_a) {
        next = __float_as_int(a1.z);
      } else if (leaf_a >= 0) {
        leaf = leaf_a;
        next = __float_as_int(a1.z);
      } else if (!slab_hit(b0, b1, ix, iy, iz, oix, oiy, oiz, tlo, tmax)) {
        next = __float_as_int(b1.z);
      } else if (leaf_b >= 0) {
        leaf = leaf_b;
        next = __float_as_int(b1.z);
      } else {
        next = node + 2;
      }
      cs.boxes += 1u + (hit_a && leaf_a < 0);  // node + 1 was tested only after an interior hit
      node = next;
    }
    if (leaf >= 0) {
      const int first = leaf >> 8, cnt = leaf & 255;
      if constexpr (kDiag) {
        ++cs.leaf_visits;
        if (first_active_lane()) ++cs.wave_leaf_trips;
      }
      const Pre32 pr = pre32_of(ox, oy, oz, A, am);
      for (int k = first; k < first + cnt; ++k) {
        const int idx = leaf_idx[k];
        if (idx == hint) continue;
        const bool ran = test_sphere(kLdsLeaves ? sv.geo(idx) : bv.leaf_geo[k], idx, ox, oy, oz,
                                     dx, dy, dz, A, bt, bi, sv.g32(idx), pr);
        cs.fp64 += ran;
        cs.pre += !ran;
      }
      tmax = tmax_up(bt - t0);
      leaf = -1;
    }
  }
}

// hittable_list::hit(r, 0, +inf) with culling, one lane (probe kernel).
__device__ __forceinline__ int world_hit_bvh(const double4* __restrict__ geo, int n,
                                             const BvhView& bv, int hint, double ox, double oy,
                                             double oz, double dx, double dy, double dz, double A,
                                             double& best_t, CullStats& cs) {
  double bt;
  int bi;
  bool trapped;
  SectionClock<false> noclk;
  const GridC gc = grid_consts(bv);
  float t0f;
  const SphereView<false> sv{geo, bv.geo32, bv.nb_rec, nullptr};
  if (!hit_quick(geo, sv, n, bv, hint, ox, oy, oz, dx, dy, dz, A, bt, bi, cs, noclk, trapped,
                 0u, gc, bv.big_idx, t0f))
  {
    int node = bv.walk0;
    hit_traverse<false, false>(bv, bv.nodes, bv.leaf_idx, sv, hint, ox, oy, oz, dx, dy, dz, A, bt,
                               bi, cs, node, 0u, (double)t0f);
  }
  best_t = bt;
  return bi;
}


// A wave's per-lane 32-bit counters -> one 64-bit atomic each into the
// block's counter set (psrt_kernels.h TraceArgs::ray_counter: [0] rays,
// [1] full FP64 sphere tests, [2] box tests, [4] pre-rejects, [5] root-box
// tests). Called converged (whole wave).
template <bool kCount>
__device__ __forceinline__ void flush_counters(unsigned long long* ctr, unsigned rays,
                                               const CullStatsT<kCount>& cs, unsigned lane) {
  constexpr int kN = kCount ? 5 : 3;
  const unsigned v[5] = {rays, (unsigned)cs.fp64, (unsigned)cs.boxes, (unsigned)cs.pre,
                         (unsigned)cs.root};
  constexpr int slot[5] = {0, 1, 2, 4, 5};
#pragma unroll
  for (int c = 0; c < kN; ++c) {
    unsigned long long w = v[c];
    for (int off = 32; off > 0; off >>= 1) w += __shfl_xor(w, off);
    if (lane == 0 && w) atomicAdd(ctr + slot[c], w);
  }
}

template <bool kBVH, bool kStamps, bool kLds, bool kCount>
__global__ __launch_bounds__(kTraceBlock, kTraceWaves) void psrt_trace(const double4* __restrict__ geo,
                                                          const double* __restrict__ inv_r,
                                                          double* __restrict__ samples,
                                                          TraceArgs a, BvhView bv) {
  const unsigned lane = lane_id();
  const uint64_t total = a.total_units;

  // BVH nodes staged in LDS when they fit (lds_layout; host: lds_max); the walk's
  // dependent node loads then see LDS latency instead of L1/L2 latency
  // With kLds, the spheres (geo, 1/r) are staged as well: the per-lane gathers
  // (previous-hit test, grid cell items, the hit record) then read LDS.
  // (dynamic LDS, sized by the host for this scene: psrt_kernels.h lds_layout)
  extern __shared__ __attribute__((aligned(16))) unsigned char s_dyn[];
  const LdsLayout lay = lds_layout(a.n, bv.n_nodes, bv.n_leaf, bv.n_big);
  float4* const s_nodes = (float4*)(s_dyn + lay.nodes);
  LdsSphere* const s_sph = (LdsSphere*)(s_dyn + lay.sph);
  int* const s_leaf = (int*)(s_dyn + lay.leaf);
  int* const s_big = (int*)(s_dyn + lay.big);
  // Constants only the refill block reads (camera basis, image size, the
  // divisions' magic numbers, the seed) live in LDS and are re-read on every
  // refill through an offset the compiler cannot see through: held across
  // the loop they would take ~40 registers and spill to scratch.
  __shared__ RefillConst s_rc;
  __shared__ GridC s_gc;
  // counters flushed from the lanes (refill block): rays, then (counting
  // variant) the tests by kind, in the counter-set order
  constexpr unsigned kFlushWords = kCount ? 6 : 3;
  __shared__ unsigned long long s_flush[kFlushWords];
  if (threadIdx.x < kFlushWords) s_flush[threadIdx.x] = 0ull;
  if (threadIdx.x == 0) s_gc = grid_consts(bv);
  if (threadIdx.x < 12)
    s_rc.cam[threadIdx.x] = threadIdx.x < 3   ? a.org[threadIdx.x]
                            : threadIdx.x < 6 ? a.llc[threadIdx.x - 3]
                            : threadIdx.x < 9 ? a.hor[threadIdx.x - 6]
                                              : a.ver[threadIdx.x - 9];
  if (threadIdx.x < kMaxFrames) s_rc.seedmix[threadIdx.x] = a.seedmix[threadIdx.x];
  if (threadIdx.x <= kQueuePhases) s_rc.ph_first[threadIdx.x] = a.ph_first[threadIdx.x];
  if (threadIdx.x < kQueuePhases) {
    s_rc.ph_base[threadIdx.x] = a.ph_base[threadIdx.x];
    s_rc.ph_size[threadIdx.x] = a.ph_size[threadIdx.x];
  }
  if (threadIdx.x == 0) {
    s_rc.wm1 = (double)(a.width - 1);
    s_rc.hm1 = (double)(a.height - 1);
    s_rc.rwm1 = a.width > 1 ? 1.0 / s_rc.wm1 : 0.0;
    s_rc.rhm1 = a.height > 1 ? 1.0 / s_rc.hm1 : 0.0;
    s_rc.div_s = a.div_s;
    s_rc.div_w = a.div_w;
    s_rc.div_p = a.div_p;
    s_rc.frames = a.frames;
    s_rc.hm1_i = a.height - 1;
    s_rc.row_offset = a.row_offset;
    s_rc.row_stride = a.row_stride;
    s_rc.s_begin = a.s_begin;
    // one workgroup in kDrainEvery stores the drain flag: every store goes
    // to the same host-visible word, and 12k of them (one per wave) queued
    // behind each other cost ~1 ms per launch (profiles/r06_drain)
    s_rc.drain_flag = blockIdx.x % kDrainEvery == 0 ? a.drain_flag : nullptr;
    s_rc.drain_epoch = a.drain_epoch;
  }
  if constexpr (kLds) {  // the host sized the dynamic LDS by lds_layout
    for (int e = threadIdx.x; e < 2 * (bv.n_nodes + 1); e += blockDim.x) s_nodes[e] = bv.nodes[e];
    for (int e = threadIdx.x; e < a.n; e += blockDim.x) {
      s_sph[e].geo = geo[e];
      s_sph[e].g32 = bv.geo32[e];
      s_sph[e].nb = bv.nb_rec[e];
      s_sph[e].inv = inv_r[e];
    }
    for (int e = threadIdx.x; e < bv.n_leaf; e += blockDim.x) s_leaf[e] = bv.leaf_idx[e];
    for (int e = threadIdx.x; e < bv.n_big; e += blockDim.x) s_big[e] = bv.big_idx[e];
  }
  __syncthreads();
  const float4* __restrict__ nodes = kLds ? s_nodes : bv.nodes;
  const int* __restrict__ lleaf = kLds ? s_leaf : bv.leaf_idx;
  SphereView<kLds> sv;
  if constexpr (kLds) sv.s = s_sph;
  else sv = SphereView<false>{geo, bv.geo32, bv.nb_rec, inv_r};
  const int* __restrict__ lbig = kLds ? s_big : bv.big_idx;

  // wave-uniform work window
  uint64_t win_base = 0;
  unsigned win_left = 0;
  bool exhausted = false;
  bool tailp = false;  // exhausted, and the launch's tail runs at kTailPrio (a.tail_prio)

  bool active = false;
  bool done = false;  // sample finished; its colour is stored by the next refill block
  double ox = 0, oy = 0, oz = 0, dx = 0, dy = 0, dz = 0, A = 0;
  int k = 0;          // bounces (hits) so far: current trace is at depth max_depth-k
  uint64_t rng = 0;
  unsigned q = 0;     // pixel index within the shard
  unsigned su = 0;    // this sample's unit (q * s_count + sample index in the chunk)
  unsigned rays = 0;  // the reference rays of this lane's trapped paths (§9); traced ones: `traced`
  int hint = -1;  // sphere the ray starts on (the previous hit), tested first
  bool pending = false;  // parked for the next batched BVH pass
  unsigned wbox0 = 0;    // diagnostic build: box tests before this ray's walk
  bool wfin = false;     // diagnostic build: the parked ray had a finite bound
  int wnode = 0;         // where the parked ray's walk resumes
  float wt0 = 0.0f;      // its re-basing point: the root-box entry of a far origin (hit_quick), else 0
  bool sc_wait = false;  // hit resolved (pbi, pbt), scatter waits for a queued trial
  // look-ahead of random_in_unit_sphere (vec3.h:83-95): accepted trials, in
  // stream order, as raw rand() triples (z, y, x draw order)
  uint32_t q0x = 0, q0y = 0, q0z = 0, q1x = 0, q1y = 0, q1z = 0;
  bool qv0 = false, qv1 = false;  // slot 0 / slot 1 of the queue hold a trial
  double pbt = 0.0;      // closest t / index so far of this ray's world.hit
  int pbi = -1;
  CullStatsT<kCount> cs{};
  unsigned long long traced = 0;  // wave-uniform: rays this wave traced
  SectionClock<kStamps> clk;
  __shared__ unsigned s_util[kStamps ? 2 * kUCount : 1];
  if constexpr (kStamps) {
    for (int e = threadIdx.x; e < 2 * kUCount; e += blockDim.x) s_util[e] = 0u;
    __syncthreads();
    clk.ucnt = s_util;
  }
  clk.start();
  unsigned long long* wlog = nullptr;  // diagnostic build: this wave's timeline
  unsigned iters = 0;                   // diagnostic build: loop iterations of this wave
  if constexpr (kStamps) {
    if (a.wave_log) {
      wlog = a.wave_log + 5 * (size_t)(blockIdx.x * (kTraceBlock / 64) + threadIdx.x / 64);
      const unsigned long long t = __builtin_amdgcn_s_memrealtime();
      if (lane == 0) wlog[0] = t, wlog[1] = 0;
    }
  }

  for (;;) {
    // ---- finish + refill lanes whose sample ended (wavefront ballot compaction) ----
    // The block runs for the wave once at least refill_min lanes are idle (or
    // none is live): its cost is per wave, so batching finished lanes pays
    // for the few iterations they sit idle.
    const bool need = !active;
    const uint64_t need_mask = __ballot(need);
    const bool run_block = need_mask != 0 && ((unsigned)__popcll(need_mask) >= kRefillMin ||
                                              need_mask == __ballot(1));
    if (run_block) {
      // The per-lane counters are 32-bit. Between two runs of this block a lane
      // adds at most one sample's work (it idles once its sample ends), which the
      // host bounds below 2^32 - a.flush_at: flush them to the 64-bit totals
      // once any lane's reaches a.flush_at (tests set it low to run this path).
      if (__builtin_expect(__ballot(max(rays, max(max((unsigned)cs.fp64, (unsigned)cs.boxes),
                                                  max((unsigned)cs.pre, (unsigned)cs.root))) >=
                                    a.flush_at) != 0, 0)) {
        atomicAdd(&s_flush[0], (unsigned long long)rays);  // LDS; to HBM at exit
        atomicAdd(&s_flush[1], (unsigned long long)cs.fp64);
        atomicAdd(&s_flush[2], (unsigned long long)cs.boxes);
        if constexpr (kCount) {
          atomicAdd(&s_flush[4], (unsigned long long)cs.pre);
          atomicAdd(&s_flush[5], (unsigned long long)cs.root);
        }
        rays = 0u;
        cs.fp64 = cs.boxes = cs.pre = cs.root = 0u;
      }
      // sky (main.cc:46-48) x 0.5^k, or black; store
      [[maybe_unused]] const bool stored = done;
      if (done) {
        // The colour is a function of (t, k) alone (sample_colour): store those
        // (10 B) in unit order. A wave's window is a run of consecutive units,
        // so its stores fill whole lines in its XCD's L2 before write-back.
        clk.util(kUStore);
        double tt = 0.0;
        unsigned short kk = kSampleBlack;
        if (pbi < 0 && a.max_depth >= 0) {
          const double y = (1.0 / sqrt_f64(A)) * dy;  // unit_vector (vec3.h:151-154)
          tt = 0.5 * (y + 1.0);
          kk = (unsigned short)(k < kSampleKCap ? k : kSampleKCap);
        }
        const unsigned u = su;  // < total < 2^32
        __builtin_nontemporal_store(tt, samples + u);
        __builtin_nontemporal_store(kk, (unsigned short*)(samples + total) + u);
        done = false;
      }
    }
    if (run_block && !exhausted) {
      const unsigned cnt = (unsigned)__popcll(need_mask);
      const unsigned rank = mbcnt64(need_mask);
      // Guided work queue (TraceArgs::ph_*): one atomicAdd per ticket; ticket
      // sizes shrink from kWorkChunk to 64 over the last few windows per wave,
      // so no wave starts a large window while the others are nearly done.
      // Every size is >= 64, so one ticket always covers the overflow.
      uint64_t nb = 0;
      unsigned wsize = kWorkChunk;
      if (cnt > win_left) {
        unsigned zq = 0;
        asm volatile("" : "+v"(zq));  // the phases are re-read from LDS here
        const RefillConst& rq = *(const RefillConst*)((const char*)&s_rc + zq);
        // sharded heads (psrt_kernels.h kQueues): this block's own head first,
        // then the next ones once it has run past the end of the work
        for (unsigned qnext = 0;; ++qnext) {
          const unsigned h = (blockIdx.x + qnext) % kQueues;
          uint64_t tk = 0;
          if (lane == 0) tk = atomicAdd(a.work_counter + kShardStride * h, 1ull);
          tk = __shfl(tk, 0) * kQueues + h;  // global ticket
          int ph = 0;
          while (ph < kQueuePhases - 1 && tk >= rq.ph_first[ph + 1]) ++ph;
          nb = rq.ph_base[ph] + (tk - rq.ph_first[ph]) * rq.ph_size[ph];
          wsize = rq.ph_size[ph];
          if (nb < total || qnext == kQueues - 1) break;
        }
      }
      if (need) {
        clk.util(kURefill);
        const uint64_t unit = rank < win_left ? win_base + rank : nb + (rank - win_left);
        if (unit < total) {  // total < 2^32 (host chunking)
          unsigned zo = 0;
          asm volatile("" : "+v"(zo));  // keeps the LDS reads below inside the loop
          const RefillConst& rc = *(const RefillConst*)((const char*)&s_rc + zo);
          const FastDiv ds = rc.div_s, dw = rc.div_w;
          q = fast_div((unsigned)unit, ds);  // f * pixels + pixel (frame-major units)
          su = (unsigned)unit;
          const unsigned sl = su - q * ds.d;
          unsigned f = 0;  // frame of a multi-frame launch (wave-uniform branch)
          if (rc.frames > 1) {
            f = fast_div(q, rc.div_p);
            q -= f * rc.div_p.d;
          }
          const unsigned row_k = fast_div(q, dw);
          const unsigned i = q - row_k * dw.d;
          const int r = rc.row_offset + (int)row_k * rc.row_stride;
          const int j = rc.hm1_i - r;
          const unsigned pix = (unsigned)j * dw.d + i;
          const unsigned s = (unsigned)rc.s_begin + sl;
          PSRT_ABLATE_AT(REFILL);
          rng = splitmix64((((uint64_t)pix) << 32 | (uint64_t)s) ^ rc.seedmix[f]);
          // main.cc:80-81, camera.h:25-28
          const double xu = (double)i + random_double(rng);
          const double xv = (double)j + random_double(rng);
          double u, v;
          if (rc.rwm1 != 0.0 && rc.rhm1 != 0.0) {  // uniform: the image is at least 2 x 2
            u = div_by(xu, rc.wm1, rc.rwm1);
            v = div_by(xv, rc.hm1, rc.rhm1);
          } else {
            u = xu / rc.wm1;
            v = xv / rc.hm1;
          }
          const double* cam = rc.cam;  // origin, lower_left, horizontal, vertical
          ox = cam[0], oy = cam[1], oz = cam[2];
          dx = ((cam[3] + u * cam[6]) + v * cam[9]) - ox;
          dy = ((cam[4] + u * cam[7]) + v * cam[10]) - oy;
          dz = ((cam[5] + u * cam[8]) + v * cam[11]) - oz;
          A = (dx * dx + dy * dy) + dz * dz;
          k = 0;
          hint = -1;
          qv0 = qv1 = false;  // the sample's stream starts here: no look-ahead yet
          active = true;
        }
      }
      if (cnt > win_left) {  // the new window serves the overflow
        win_base = nb + (cnt - win_left);
        win_left = wsize - (cnt - win_left);
      } else {
        win_base += cnt;
        win_left -= cnt;
      }
      if (win_base >= total) {
        exhausted = true;
        // Launch tail: this wave's remaining paths decide when the launch
        // (and the next frame's start on its CUs) ends; let them issue first.
        if (a.tail_prio) {
          tailp = true;
          __builtin_amdgcn_s_setprio(kTailPrio);
        }
        // the drain flag (read from LDS, a vector store): a launch waiting on
        // another stream for this one's tail may start now
#ifndef PSRT_NO_DRAIN_FLAG  // A/B builds only: without the store, rt_context_wait_drain never returns
        if (lane == 0) {
          unsigned zd = 0;
          asm volatile("" : "+v"(zd));
          const RefillConst& rd = *(const RefillConst*)((const char*)&s_rc + zd);
          unsigned long long* const fl = rd.drain_flag;
          if (fl) __hip_atomic_store(fl, rd.drain_epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
#endif
        if constexpr (kStamps) {
          const unsigned long long t = __builtin_amdgcn_s_memrealtime();
          if (wlog && lane == 0) wlog[1] = t, wlog[3] = iters;
        }
      }
    }
    clk.mark(kSecRefill);
    if (__ballot(active) == 0) break;
    if constexpr (kStamps) ++iters;

    // ---- world.hit(r, 0, inf, rec)  (main.cc:40) ----
    // Cheap part for every live, non-parked lane; rays that need the BVH walk
    // park (pending) and are walked together in one batched pass once enough
    // lanes wait (or nothing else can progress): the pass then runs at high
    // SIMD occupancy instead of once per iteration for a handful of lanes.
    bool resolved = false, finish = false;
    traced += (unsigned)__popcll(__ballot(active && !pending && !sc_wait && a.max_depth >= 0));
    __builtin_amdgcn_s_setprio(kHitPrio);
    if (active && !pending && !sc_wait) {
      if (a.max_depth < 0) {  // main.cc:36-37 at the first call: black, no trace
        finish = true;
      } else {
        // this ray is one of the reference's rays: counted in `traced` above
        // (wave-uniform), added to the ray total at exit
        clk.util(kUHit);
        if constexpr (kBVH) {
          bool trapped;
          unsigned zg = 0;
          asm volatile("" : "+v"(zg));  // re-read the grid constants from LDS here
          const GridC& gc = *(const GridC*)((const char*)&s_gc + zg);
          resolved = hit_quick(geo, sv, a.n, bv, hint, ox, oy, oz, dx, dy, dz, A, pbt, pbi,
                               cs, clk, trapped, q, gc, lbig, wt0);
          PSRT_ABLATE_AT(HIT_QUICK);
          pending = !resolved;
          wnode = bv.walk0;
          if constexpr (kStamps) {
            wbox0 = cs.boxes;
            wfin = pbt < 1e30;
          }
          if (trapped && k < a.max_depth) {
            // the reference traces the max_depth - k rays that remain, all at
            // t = +-0 on this sphere, then returns black (pbi >= 0 below)
            rays += (unsigned)(a.max_depth - k);
            finish = true;
          }
        } else {
          // small scenes (no BVH): the reference scan, plus the §9 test
          bool trapped = false;
          pbi = sweep_linear<true>(geo, a.n, ox, oy, oz, dx, dy, dz, A, 0.0, __builtin_inf(),
                                   pbt, bv.fixpoint ? hint : -1, &trapped);
          cs.fp64 += a.n;
          resolved = true;
          const double am = __builtin_fmax(__builtin_fabs(ox),
                                           __builtin_fmax(__builtin_fabs(oy), __builtin_fabs(oz)));
          if (trapped && am <= 0x1p40 && A > 0.0 && A < 1e200 && k < a.max_depth) {
            rays += (unsigned)(a.max_depth - k);
            finish = true;
          }
        }
      }
    }
    if (tailp) __builtin_amdgcn_s_setprio(kTailPrio);  // back to the base priority
    else __builtin_amdgcn_s_setprio(0);
    clk.mark(kSecHit);
    if constexpr (kBVH) {
      const uint64_t pend = __ballot(pending);
      const uint64_t movable = __ballot(active && !pending);
      if (pend != 0 && ((unsigned)__popcll(pend) >= kWalkBatch || movable == 0)) {
        __builtin_amdgcn_s_setprio(kWalkPrio);
        if (pending) {
          clk.util(kUWalk);
          PSRT_ABLATE_AT(WALK);
          hit_traverse<kStamps, kLds>(bv, nodes, lleaf, sv, hint, ox, oy,
                                                         oz, dx, dy, dz, A, pbt, pbi, cs, wnode,
                                                         movable ? kWalkTail : 0u, (double)wt0);
          if (wnode >= bv.n_nodes) {
            pending = false;
            resolved = true;
            if constexpr (kStamps) {
              const unsigned wb = cs.boxes - wbox0;
              bool big = false;
              for (int b = 0; b < bv.n_big; ++b) big = big || bv.big_idx[b] == pbi;
              clk.add(pbi < 0 ? kUWMiss : big ? kUWBig : kUWBvh, wb);
              clk.add(wfin ? kUWFin : kUWInf, wb);
            }
          }
        }
        if (tailp) __builtin_amdgcn_s_setprio(kTailPrio);
        else __builtin_amdgcn_s_setprio(0);
      }
    }
    // depth-0 hit: 0.5 * ray_color(.., -1) = black (main.cc:36-37, 43)
    if (resolved && (pbi < 0 || k >= a.max_depth)) finish = true;
    const int hit = pbi;
    const double t = pbt;
    clk.mark(kSecTraverse);

    // ---- random_in_unit_sphere look-ahead (vec3.h:83-95) ----
    // Each sample draws from its own stream, so the trials of its next bounces
    // can be generated early, in stream order, and queued; a lane that ends its
    // sample just drops its queue (those draws would never have been made, and
    // no other sample's stream depends on them). Every live lane tops up its
    // queue each iteration, converged; the loop runs at most rng_extra more
    // trials while a lane that scatters now has nothing queued. A lane still
    // without a trial then keeps its resolved hit and scatters in a later
    // iteration (sc_wait): its draws stay in stream order either way.
    const bool want = (resolved && !finish) || sc_wait;
    PSRT_ABLATE_AT(TRIALS);
    {
      const bool can_fill = active && !finish;
      // branch-free body: every lane computes a trial; only lanes with room
      // take it (their stream advances), so the draws stay in stream order
      int f = 0;
      do {
        const bool go = can_fill && !qv1;
        if (go) clk.util(kUTrial);
        uint32_t z, y, x;
        uint64_t nxt;
        raw32_x3(rng, z, y, x, nxt);  // z, y, x: g++'s draw order (vec3.h:78-81); raw outputs
        const bool in = in_unit_sphere_raw_f32(x, y, z);  // FP64 only near the surface
        rng = go ? nxt : rng;
        const bool push = go && in;
        const bool to0 = push && !qv0, to1 = push && qv0;
        q0x = to0 ? x : q0x, q0y = to0 ? y : q0y, q0z = to0 ? z : q0z;
        q1x = to1 ? x : q1x, q1y = to1 ? y : q1y, q1z = to1 ? z : q1z;
        qv1 = qv1 || to1;
        qv0 = qv0 || to0;
        ++f;
      } while (f < kRngFill ||
               (f < kRngFill + kRngExtra &&
                __ballot(want && !qv0) != 0));
    }
    clk.mark(kSecFillShade);

    // ---- scatter: target = (p + n) + random_in_hemisphere(n)  (main.cc:42-43) ----
    const bool have = qv0;
    sc_wait = want && !have;
    PSRT_ABLATE_AT(SCATTER);
    if (want && have) {
      clk.util(kUScatter);
      const HitRec h = hit_record_of(sv.geo(hit), sv.inv(hit), t, ox, oy, oz, dx, dy, dz);
      // vec3.h:78-81 random(-1, 1) from the queued draws; vec3.h:102-109 flip
      double rx = pm1_raw(q0x), ry = pm1_raw(q0y), rz = pm1_raw(q0z);
      q0x = q1x, q0y = q1y, q0z = q1z;
      qv0 = qv1;
      qv1 = false;
      if (!((rx * h.nx + ry * h.ny) + rz * h.nz > 0.0)) rx = -rx, ry = -ry, rz = -rz;
      dx = ((h.px + h.nx) + rx) - h.px;
      dy = ((h.py + h.ny) + ry) - h.py;
      dz = ((h.pz + h.nz) + rz) - h.pz;
      ox = h.px, oy = h.py, oz = h.pz;
      A = (dx * dx + dy * dy) + dz * dz;
      hint = hit;
      ++k;
    }
    clk.mark(kSecScatter);

    // ---- sample done: colour and store in the next finish + refill block ----
    if (finish) {
      done = true;
      active = false;
    }
    clk.mark(kSecFillShade);
  }
  if constexpr (kStamps) {
    if (wlog) {
      const unsigned long long t = __builtin_amdgcn_s_memrealtime();
      if (lane == 0) wlog[2] = t, wlog[4] = iters;
    }
    if (lane == 0)
      for (int k2 = 0; k2 < kSecCount; ++k2) atomicAdd(a.stamps + k2, (unsigned long long)clk.acc[k2]);
    // wave-level counters live in whichever lane was first active: sum them all
    atomicAdd(a.stamps + 8, (unsigned long long)cs.wave_trips);
    atomicAdd(a.stamps + 9, (unsigned long long)cs.wave_leaf_trips);
    atomicAdd(a.stamps + 10, (unsigned long long)cs.trav_rays);
    atomicAdd(a.stamps + 11, (unsigned long long)cs.leaf_visits);
    __syncthreads();  // every wave of the block has left the loop
    for (int e = threadIdx.x; e < 2 * kUCount; e += blockDim.x)
      atomicAdd(a.stamps + 12 + e, (unsigned long long)s_util[e]);
  }

  unsigned long long* const ctr = a.ray_counter + kShardStride * (blockIdx.x % kQueues);
  flush_counters(ctr, rays, cs, lane);
  if (lane == 0 && traced) {
    atomicAdd(ctr, traced);      // the traced rays (the lanes' counters hold the trapped rest)
    atomicAdd(ctr + 3, traced);  // rays_traced
  }
  __syncthreads();  // every wave of the block has left the loop (and flushed to LDS)
  if (threadIdx.x < kFlushWords && threadIdx.x != 3 && s_flush[threadIdx.x])
    atomicAdd(ctr + threadIdx.x, s_flush[threadIdx.x]);
}

#define PSRT_INSTANTIATE1(B, S, L, C)                                                       \
  template __global__ void psrt_trace<B, S, L, C>(const double4* __restrict__,               \
                                                  const double* __restrict__,                \
                                                  double* __restrict__, TraceArgs, BvhView);
#define PSRT_INSTANTIATE(B, S, L) PSRT_INSTANTIATE1(B, S, L, false) PSRT_INSTANTIATE1(B, S, L, true)
PSRT_INSTANTIATE(false, false, false)
PSRT_INSTANTIATE(true, false, false)
PSRT_INSTANTIATE(true, false, true)
PSRT_INSTANTIATE(false, true, false)
PSRT_INSTANTIATE(true, true, false)
PSRT_INSTANTIATE(true, true, true)
#undef PSRT_INSTANTIATE
#undef PSRT_INSTANTIATE1

// pixel_color += sample, in sample order (main.cc:77-84); write_color on the
// last chunk (color.h:8-24).

// Frame blockIdx.y's records and outputs; block 0 of frame 0 folds the trace
// launch's counter sets and re-zeroes them and the queue heads.
__device__ __forceinline__ void reduce_prologue(ReduceArgs& a) {
  if (blockIdx.y > 0) {  // frame blockIdx.y of a multi-frame launch
    const size_t f = blockIdx.y;
    a.samp_t += f * a.frame_units;
    a.samp_k += f * a.frame_units;
    if (a.accum) a.accum += f * a.accum_stride;
    if (a.rgb8) a.rgb8 += f * a.rgb8_stride;
    a.fold_stats = 0;
  }
  // the trace launch's sharded counter sets -> totals (-> host), then the
  // sets and queue heads back to zero (ReduceArgs; stream order puts this
  // after every trace block and before the context's next launch)
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
}

// write_color (color.h:8-24) of one pixel's sums: 3 bytes in the low 24 bits
__device__ __forceinline__ unsigned write_color_bytes(double r, double g, double b, double inv) {
  const double c[3] = {r, g, b};
  unsigned v = 0;
#pragma unroll
  for (int ch = 0; ch < 3; ++ch) {
    double x = __builtin_sqrt(c[ch] * inv);
    x = (x < 0.0) ? 0.0 : x;  // std::max(x, 0.0)
    x = (0.999 < x) ? 0.999 : x;  // std::min(x, 0.999)
    v |= (unsigned)(unsigned char)(int)(255.999 * x) << (8 * ch);
  }
  return v;
}

__global__ __launch_bounds__(kReduceBlock) void psrt_reduce(ReduceArgs a) {
  reduce_prologue(a);
  // One wave per 64 pixels. A pixel's samples are contiguous, so the wave
  // stages [64 pixels][kReduceTile samples] tiles through LDS, then each lane
  // adds its pixel's samples in order.
  __shared__ __attribute__((aligned(16))) double s_t[kReduceBlock][kReduceTile + 2];
  __shared__ __attribute__((aligned(16))) unsigned short s_k[kReduceBlock][kReduceTile + 4];
  const unsigned lane = threadIdx.x;
  const unsigned q0 = blockIdx.x * kReduceBlock;
  const unsigned q = q0 + lane;
  const unsigned S = (unsigned)a.s_count;
  double r = 0.0, g = 0.0, b = 0.0;
  // this lane's sums (ReduceArgs::accum_pitch: rows may lie apart)
  double* const acc_q =
      !a.accum ? nullptr
      : a.accum_pitch ? a.accum + (size_t)(q / a.width) * a.accum_pitch + (size_t)(q % a.width) * 3
                      : a.accum + (size_t)q * 3;
  if (!a.first_chunk && q < a.pixels) {
    r = acc_q[0];
    g = acc_q[1];
    b = acc_q[2];
  }
  // Tiles of a pixel run: kReduceTile doubles of t and kReduceTile uint16 of
  // k per pixel. With s_count % 4 == 0 they are 16-B aligned: t is read in
  // 16-B pieces (kLT lanes per pixel), k in 8-B pieces (kLK lanes per pixel),
  // and the next tile's loads are in flight while this tile is summed from
  // LDS; else element by element.
  constexpr int kLT = kReduceTile / 2, kPT = 64 / kLT;  // t: lanes, pixels per load
  constexpr int kLK = kReduceTile / 4, kPK = 64 / kLK;  // k: lanes, pixels per load
  static_assert(kReduceBlock == 64 && (kReduceTile == 16 || kReduceTile == 32),
                "tile shape of the loads below");
  auto sum_tile = [&](unsigned T) {
    if (a.fast_k) {
      // every k < 1000: sample_colour's operations, with 0.5^k as one ldexp
      // (exact: the sky is >= 0.5) and black as a select, not a branch; a
      // black sample adds +0.0, as there
      for (unsigned j = 0; j < T; ++j) {
        const double tt = s_t[lane][j];
        const unsigned kk = s_k[lane][j];
        const bool blk = kk == kSampleBlack;
        const double w = 1.0 - tt;
        const double cr = __builtin_ldexp(w + tt * 0.5, -(int)kk);
        const double cg = __builtin_ldexp(w + tt * 0.7, -(int)kk);
        const double cb = __builtin_ldexp(w + tt * 1.0, -(int)kk);
        r += blk ? 0.0 : cr;
        g += blk ? 0.0 : cg;
        b += blk ? 0.0 : cb;
      }
      return;
    }
    for (unsigned j = 0; j < T; ++j) {
      double cr, cg, cb;
      sample_colour(s_t[lane][j], s_k[lane][j], cr, cg, cb);
      r += cr;
      g += cg;
      b += cb;
    }
  };
  if (S % 4 == 0) {
    auto load = [&](unsigned s0, double2* vt, uint2* vk) {
      const unsigned T = min((unsigned)kReduceTile, S - s0);
#pragma unroll
      for (int i = 0; i < kLT; ++i) {
        const unsigned p = kPT * i + lane / kLT, j = (lane % kLT) * 2;
        vt[i] = make_double2(0.0, 0.0);
        if (q0 + p < a.pixels && j < T) {
          vt[i] = *(const double2*)(a.samp_t + (size_t)(q0 + p) * S + s0 + j);
        }
      }
#pragma unroll
      for (int i = 0; i < kLK; ++i) {
        const unsigned p = kPK * i + lane / kLK, j = (lane % kLK) * 4;
        vk[i] = make_uint2(0u, 0u);
        if (q0 + p < a.pixels && j < T) {
          vk[i] = *(const uint2*)(a.samp_k + (size_t)(q0 + p) * S + s0 + j);
        }
      }
    };
    auto stage = [&](const double2* vt, const uint2* vk) {
      __syncthreads();
#pragma unroll
      for (int i = 0; i < kLT; ++i)
        *(double2*)&s_t[kPT * i + lane / kLT][(lane % kLT) * 2] = vt[i];
#pragma unroll
      for (int i = 0; i < kLK; ++i)
        *(uint2*)&s_k[kPK * i + lane / kLK][(lane % kLK) * 4] = vk[i];
      __syncthreads();
    };
    // kReduceInFlight tiles in flight (a ring in registers): the loads are
    // latency-bound at this occupancy (the LDS tiles allow ~7 waves per CU);
    // 1 -> 2 tiles: 4.1 -> 3.7 ms per 20 C3 frames (profiles/r04_reduce3)
    constexpr unsigned kNT = kReduceInFlight, kT = kReduceTile;
    double2 vt[kNT][kLT];
    uint2 vk[kNT][kLK];
#pragma unroll
    for (unsigned b = 0; b < kNT; ++b)
      if (b * kT < S) load(b * kT, vt[b], vk[b]);
    for (unsigned s0 = 0; s0 < S; s0 += kNT * kT) {
#pragma unroll
      for (unsigned b = 0; b < kNT; ++b) {
        const unsigned sb = s0 + b * kT;
        if (sb >= S) break;  // block-uniform
        stage(vt[b], vk[b]);
        if (sb + kNT * kT < S) load(sb + kNT * kT, vt[b], vk[b]);  // refill this slot
        sum_tile(min(kT, S - sb));
      }
    }
  } else {
    for (unsigned s0 = 0; s0 < S; s0 += kReduceTile) {
      const unsigned T = min((unsigned)kReduceTile, S - s0);
      constexpr int kPP = 64 / kReduceTile;  // pixels per load
      double vt[8];
      unsigned short vk[8];
      for (int h = 0; h < kReduceTile / 8; ++h) {
        __syncthreads();
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const unsigned p = 8 * kPP * h + kPP * i + lane / kReduceTile, j = lane % kReduceTile;
          const bool ok = q0 + p < a.pixels && j < T;
          const size_t u = (size_t)(q0 + p) * S + s0 + j;
          vt[i] = ok ? a.samp_t[u] : 0.0;
          vk[i] = ok ? a.samp_k[u] : (unsigned short)0;
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          s_t[8 * kPP * h + kPP * i + lane / kReduceTile][lane % kReduceTile] = vt[i];
          s_k[8 * kPP * h + kPP * i + lane / kReduceTile][lane % kReduceTile] = vk[i];
        }
      }
      __syncthreads();
      sum_tile(T);
    }
  }
  if (a.accum && q < a.pixels) {
    acc_q[0] = r;
    acc_q[1] = g;
    acc_q[2] = b;
  }
  if (a.rgb8) {  // write_color (color.h:8-24)
    __shared__ __attribute__((aligned(16))) unsigned char s_rgb[kReduceBlock * 3];
    const double inv = 1.0 / (double)a.spp_total;
    const double c[3] = {r, g, b};
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) {
      double x = __builtin_sqrt(c[ch] * inv);
      x = (x < 0.0) ? 0.0 : x;  // std::max(x, 0.0)
      x = (0.999 < x) ? 0.999 : x;  // std::min(x, 0.999)
      s_rgb[lane * 3 + ch] = (unsigned char)(int)(255.999 * x);
    }
    __syncthreads();
    // The wave's pixels are 192 contiguous bytes: written as 12 x 16-B stores
    // (the frame may be pinned host memory, written across the link: the
    // frame's device-to-host transfer then needs no copy of its own)
    const unsigned nb = min((unsigned)kReduceBlock, a.pixels - q0) * 3u;
    if (!a.rgb8_pitch) {
      unsigned char* const dst = a.rgb8 + (size_t)q0 * 3;
      if (nb == kReduceBlock * 3u && ((uintptr_t)dst & 15u) == 0) {
        if (lane < kReduceBlock * 3 / 16) ((uint4*)dst)[lane] = ((const uint4*)s_rgb)[lane];
      } else {
        for (unsigned e = lane; e < nb; e += kReduceBlock) dst[e] = s_rgb[e];
      }
    } else {
      // rows rgb8_pitch apart (another shard's rows between them): each byte
      // to its row; a wave's bytes stay contiguous within a row, so the
      // stores still coalesce
      for (unsigned e = lane; e < nb; e += kReduceBlock) {
        const unsigned qq = q0 + e / 3;
        a.rgb8[(size_t)(qq / a.width) * a.rgb8_pitch + (size_t)(qq % a.width) * 3 + e % 3] =
            s_rgb[e];
      }
    }
  }
}

// psrt_reduce beside a resident trace (frames in flight). A
// psrt_trace launch holds 6 waves per SIMD at 80 VGPRs and ~150 KB of LDS per
// CU, and its SGPRs (106, rounded up, plus the trap handler's 16) leave room
// for one more wave per SIMD only if that wave needs at most 16 SGPRs, 32
// VGPRs and no LDS (measured: scripts/coresident_probe.py, profiles/r06_drain).
// psrt_reduce (252 VGPRs, 22 KB of LDS) waits for a free slot until the next
// frame's trace drains; this variant starts at once beside it. To fit:
//  - its arguments are read through a pointer held in a VGPR, so every value
//    derived from them is per-lane; the few it branches or loops on are made
//    scalar one at a time (readfirstlane);
//  - no lane is masked off: a lane past the last pixel takes the last pixel
//    and stores the same bytes there as its owner (identical values);
//  - no statistics fold (the host launches psrt_reduce for a fold).
// A lane per pixel reads its own records, four samples per step (32 B of t,
// 8 B of k), and adds them in psrt_reduce's order with its operations:
// bit-identical. fast_k and s_count % 4 == 0 only.
#ifndef PSRT_LEAN_PRIO
#define PSRT_LEAN_PRIO 0  // issue priority of psrt_reduce_lean's waves (0 / 1 / 3: profiles/r06_drain)
#endif

template <class T>
__device__ __forceinline__ T uniform(T v) {  // a wave-uniform value into one SGPR
  return (T)__builtin_amdgcn_readfirstlane((int)v);
}

__global__ __launch_bounds__(kReduceBlock) void psrt_reduce_lean(ReduceArgs) {
  // the trace beside it runs at priority 1-3 in most sections; a reduce wave
  // at 0 still finishes within the trace (0.6 ms) and takes the fewest issue
  // slots from it: C3 two in flight 11.83 ms per frame at 0, 11.87 at 1,
  // 11.88 at 3 (profiles/r06_drain)
  __builtin_amdgcn_s_setprio(PSRT_LEAN_PRIO);
  uintptr_t ka = (uintptr_t)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+v"(ka));  // the argument block's address in a VGPR
  const ReduceArgs* const ap = (const ReduceArgs*)ka;
  const unsigned lane = threadIdx.x;
  const unsigned f = blockIdx.y;
  const unsigned pixels = ap->pixels;
  if (uniform(pixels) == 0) return;  // (the host launches no empty reduce; kept exact anyway)
  const unsigned q0 = blockIdx.x * kReduceBlock;
  const unsigned q = min(q0 + lane, pixels - 1);  // past the end: the last pixel again
  const unsigned S = (unsigned)ap->s_count;
  const unsigned width = ap->width;
  // this lane's sums: element offsets (< 2^32: a launch's frames fit in memory)
  const size_t apitch = ap->accum_pitch;
  const unsigned aoff = (unsigned)(f * ap->accum_stride) +
                        (apitch ? (q / width) * (unsigned)apitch + (q % width) * 3 : q * 3);
  double* const acc_q = ap->accum + aoff;
  double r = 0.0, g = 0.0, b = 0.0;
  if (uniform(ap->first_chunk) == 0) {
    r = acc_q[0];
    g = acc_q[1];
    b = acc_q[2];
  }
  const unsigned ro = f * (unsigned)ap->frame_units + q * S;
  const double2* const tp = (const double2*)(ap->samp_t + ro);
  const uint2* const kp = (const uint2*)(ap->samp_k + ro);
  auto add = [&](double tt, unsigned kk) {
    // psrt_reduce's operations, one channel at a time (fewer live registers)
    const bool blk = kk == kSampleBlack;
    const double w = 1.0 - tt;
    r += blk ? 0.0 : __builtin_ldexp(w + tt * 0.5, -(int)kk);
    __builtin_amdgcn_sched_barrier(0);
    g += blk ? 0.0 : __builtin_ldexp(w + tt * 0.7, -(int)kk);
    __builtin_amdgcn_sched_barrier(0);
    b += blk ? 0.0 : __builtin_ldexp(w + tt * 1.0, -(int)kk);
    __builtin_amdgcn_sched_barrier(0);
  };
  const unsigned steps = uniform(S / 4);
#pragma unroll 1
  for (unsigned st = 0; st < steps; ++st) {
    const uint2 kk = kp[st];
    const double2 t0 = tp[2 * st];
    add(t0.x, kk.x & 0xffffu);
    add(t0.y, kk.x >> 16);
    const double2 t1 = tp[2 * st + 1];
    add(t1.x, kk.y & 0xffffu);
    add(t1.y, kk.y >> 16);
  }
  if (uniform(ap->accum != nullptr)) {
    acc_q[0] = r;
    acc_q[1] = g;
    acc_q[2] = b;
  }
  if (uniform(ap->rgb8 != nullptr)) {  // write_color (color.h:8-24)
    double inv = ap->inv_spp, hi = 0.999, sc = 255.999;
    asm volatile("" : "+v"(hi), "+v"(sc));  // constants in VGPRs, not SGPR pairs
    unsigned v = 0;
    const double c[3] = {r, g, b};
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) {
      double x = __builtin_sqrt(c[ch] * inv);
      x = (x < 0.0) ? 0.0 : x;  // std::max(x, 0.0)
      x = (hi < x) ? hi : x;    // std::min(x, 0.999)
      v |= (unsigned)(unsigned char)(int)(sc * x) << (8 * ch);
      __builtin_amdgcn_sched_barrier(0);
    }
    const size_t rpitch = ap->rgb8_pitch;
    unsigned char* const rgb = ap->rgb8 + f * ap->rgb8_stride;
    unsigned char* const dst = rgb + (size_t)q0 * 3;
    if (uniform(!rpitch && q0 + kReduceBlock <= pixels && ((uintptr_t)dst & 3u) == 0)) {
      // the wave's 192 bytes as 48 dwords: dword l holds bytes 4l .. 4l + 3,
      // from pixels 4l / 3 and the next (lane shuffles, no LDS allocation);
      // lanes 48-63 store dword 47 again
      const unsigned l = min(lane, (unsigned)kReduceBlock * 3 / 4 - 1);
      const unsigned p0 = 4u * l / 3u;
      const unsigned v0 = __shfl(v, p0), v1 = __shfl(v, min(p0 + 1, (unsigned)kReduceBlock - 1));
      const uint64_t st = (uint64_t)v0 | ((uint64_t)v1 << 24);
      ((unsigned*)dst)[l] = (unsigned)(st >> (8 * ((4u * l) % 3u)));
    } else {
      unsigned char* const px = rgb + (rpitch ? (q / width) * (unsigned)rpitch + (q % width) * 3
                                              : q * 3);
      px[0] = (unsigned char)v;
      px[1] = (unsigned char)(v >> 8);
      px[2] = (unsigned char)(v >> 16);
    }
  }
}

// reduce_prologue's statistics fold for psrt_reduce_lean's launches, in the
// same register budget (arguments through a VGPR pointer): one wave.
__global__ __launch_bounds__(64) void psrt_fold_stats(ReduceArgs) {
  __builtin_amdgcn_s_setprio(3);  // 5 us, and the reduce waits for it
  uintptr_t ka = (uintptr_t)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+v"(ka));
  const ReduceArgs* const ap = (const ReduceArgs*)ka;
  const unsigned t = threadIdx.x;
  if (t < kStatWords) {
    unsigned long long* const sets = ap->sets;
    unsigned long long v = ap->first_chunk ? 0ull : ap->totals[t];
#pragma unroll
    for (int h = 0; h < kQueues; ++h) {
      v += sets[kShardStride * h + t];
      sets[kShardStride * h + t] = 0ull;
    }
    ap->totals[t] = v;
    unsigned long long* const hs = ap->host_stats;
    if (hs) hs[t] = v;
  }
  if (t < kQueues) ap->heads[kShardStride * t] = 0ull;
}

// ---- camera-ray candidate lists ------------------------------
//
// Every camera ray of pixel (i, j) has direction d = ((llc + u*h) + v*vv) - o
// (camera.h:25-28) with u in [i/(W-1), (i+1)/(W-1)], v in [j/(H-1), (j+1)/(H-1)]
// (main.cc:80-81): a parallelogram of directions, inside the cone around the
// pixel centre's direction whose half-angle reaches the four corners (the
// angle to the axis is quasi-convex, so its maximum is at a corner). A BVH
// sphere can return an accepted root only if its padded ball (r + pad, the
// same pad that bounds the root error for the BVH boxes) meets that cone. The
// cone test below is done in FP64 with the angle widened by 1e-9 rad and the
// radius by 2^-20, margins far above its own rounding (~1e-15). Camera rays
// then test the big spheres and the pixel's list only.

__device__ __forceinline__ void cam_dir(const CamListArgs& a, double u, double v, double d[3]) {
#pragma unroll
  for (int k = 0; k < 3; ++k) d[k] = ((a.llc[k] + u * a.hor[k]) + v * a.ver[k]) - a.org[k];
}

struct Cone {
  double ax, ay, az, ca, sa;  // unit axis, cos / sin of the (widened) half-angle
  bool ok;
};

__device__ __forceinline__ Cone cam_cone(const CamListArgs& a, double u0, double u1, double v0,
                                         double v1) {
  Cone c;
  double d[3];
  cam_dir(a, 0.5 * (u0 + u1), 0.5 * (v0 + v1), d);
  const double il = 1.0 / __builtin_sqrt((d[0] * d[0] + d[1] * d[1]) + d[2] * d[2]);
  c.ax = d[0] * il, c.ay = d[1] * il, c.az = d[2] * il;
  double cmin = 1.0;
  const double us[2] = {u0, u1}, vs[2] = {v0, v1};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    cam_dir(a, us[e & 1], vs[e >> 1], d);
    const double l = __builtin_sqrt((d[0] * d[0] + d[1] * d[1]) + d[2] * d[2]);
    cmin = __builtin_fmin(cmin, ((c.ax * d[0] + c.ay * d[1]) + c.az * d[2]) / l);
  }
  c.ca = cmin - 1e-9;  // cos(alpha + delta) >= cos(alpha) - delta: widens by >= 1e-9 rad
  c.sa = __builtin_sqrt(__builtin_fmax(0.0, 1.0 - c.ca * c.ca));
  c.ok = c.ca > 0.1 && il > 0.0 && il < 1e300;  // narrow, finite cone (else: no lists)
  return c;
}

// Does the ball (centre s.xyz, radius sqrt(s.w) + pad) meet the cone with apex o?
__device__ __forceinline__ bool cone_meets(const Cone& c, const CamListArgs& a, const double4 s) {
  const double cx = s.x - a.org[0], cy = s.y - a.org[1], cz = s.z - a.org[2];
  const double l2 = (cx * cx + cy * cy) + cz * cz;
  const double R = (__builtin_sqrt(s.w) + a.pad) * (1.0 + 0x1p-20);
  if (!(l2 > R * R * (1.0 + 0x1p-20))) return true;  // apex inside / near the ball (or NaN)
  const double l = __builtin_sqrt(l2);
  const double cb = ((c.ax * cx + c.ay * cy) + c.az * cz) / l;
  if (cb >= c.ca) return true;  // centre inside the cone
  const double sb = __builtin_sqrt(__builtin_fmax(0.0, 1.0 - cb * cb));
  // angle(axis, centre) - alpha must be <= asin(R / l) (<= pi/2)
  const double cosd = cb * c.ca + sb * c.sa, sind = sb * c.ca - cb * c.sa;
  return cosd >= 0.0 && sind <= R / l;
}

__global__ __launch_bounds__(64) void psrt_camera_lists(CamListArgs a) {
  __shared__ int s_tile[kCamTileCap];
  const unsigned lane = __lane_id();
  const int x0 = blockIdx.x * kCamTile, r0 = blockIdx.y * kCamTile;
  const int x1 = min(x0 + kCamTile, a.width), r1 = min(r0 + kCamTile, a.rows);
  const int px = x0 + (int)(lane % kCamTile), rk = r0 + (int)(lane / kCamTile);
  const double iw = 1.0 / (double)(a.width - 1), ih = 1.0 / (double)(a.height - 1);
  // reference rows j = H-1-r fall as the shard row rk rises (main.cc:72)
  const int jhi = a.height - 1 - (a.row_offset + r0 * a.row_stride);
  const int jlo = a.height - 1 - (a.row_offset + (r1 - 1) * a.row_stride);
  // u, v bounds: i/(W-1) etc. widened by a relative 2^-40 (covers the rounding
  // of i + random_double() and of the division, main.cc:80-81)
  const double wid = 1.0 + 0x1p-40;
  const Cone tc = cam_cone(a, x0 * iw / wid, x1 * iw * wid, jlo * ih / wid, (jhi + 1) * ih * wid);
  int cnt = 0;
  bool over = !tc.ok;
  for (int base = 0; base < a.n_leaf && !over; base += 64) {
    const int k = base + (int)lane;
    const bool cand = k < a.n_leaf && cone_meets(tc, a, a.leaf_geo[k]);
    const uint64_t m = __ballot(cand);
    const int pos = cnt + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32),
                                                         __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
    if (cand && pos < kCamTileCap) s_tile[pos] = k;
    cnt += __popcll(m);
    if (cnt > kCamTileCap) over = true;
  }
  __syncthreads();
  if (px >= a.width || rk >= a.rows) return;
  const int j = a.height - 1 - (a.row_offset + rk * a.row_stride);
  unsigned w[4] = {kCamOverflow, 0u, 0u, 0u};
  if (!over) {
    const Cone pc = cam_cone(a, px * iw / wid, (px + 1) * iw * wid, j * ih / wid, (j + 1) * ih * wid);
    unsigned n = 0;
    bool full = !pc.ok;
    for (int e = 0; e < cnt && !full; ++e) {
      const int k = s_tile[e];
      if (!cone_meets(pc, a, a.leaf_geo[k])) continue;
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

__global__ __launch_bounds__(256) void psrt_quantize(const double* __restrict__ accum,
                                                     unsigned char* __restrict__ rgb8,
                                                     unsigned n, int spp) {
  const unsigned e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  double x = __builtin_sqrt(accum[e] * (1.0 / (double)spp));
  x = (x < 0.0) ? 0.0 : x;
  x = (0.999 < x) ? 0.999 : x;
  rgb8[e] = (unsigned char)(int)(255.999 * x);
}

// hittable_list::hit probe for known-answer tests: the same sweep and record
// code as psrt_trace, one ray per thread. rays[k] = {ox,oy,oz,dx,dy,dz,tmin,tmax};
// out[k] = {index, px, py, pz, nx, ny, nz, t, front_face}.
__global__ void psrt_probe_hit(const double4* __restrict__ geo, const double* __restrict__ inv_r,
                               int n, const double* __restrict__ rays, const int* __restrict__ hints,
                               double* __restrict__ out, unsigned count, BvhView bv, int use_bvh) {
  const unsigned k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= count) return;
  const double* r = rays + (size_t)k * 8;
  const double ox = r[0], oy = r[1], oz = r[2], dx = r[3], dy = r[4], dz = r[5];
  const double A = (dx * dx + dy * dy) + dz * dz;  // sphere.cc:9
  double t;
  int i;
  if (use_bvh && r[6] == 0.0 && r[7] == __builtin_inf()) {  // the trace kernel's call shape
    CullStats cs{};
    // hint: the sphere the ray starts on (the trace kernel's previous hit)
    const int hint = hints ? hints[k] : -1;
    i = world_hit_bvh(geo, n, bv, hint >= 0 && hint < n ? hint : -1, ox, oy, oz, dx, dy, dz, A, t,
                      cs);
  } else {
    i = sweep_linear(geo, n, ox, oy, oz, dx, dy, dz, A, r[6], r[7], t);
  }
  double* o = out + (size_t)k * 9;
  o[0] = (double)i;
  if (i >= 0) {
    const HitRec h = hit_record_of(geo[i], inv_r[i], t, ox, oy, oz, dx, dy, dz);
    o[1] = h.px, o[2] = h.py, o[3] = h.pz, o[4] = h.nx, o[5] = h.ny, o[6] = h.nz;
    o[7] = t;
    o[8] = h.front ? 1.0 : 0.0;
  }
}

// Numerics probe: the f64 primitives the parity argument rests on.
__global__ void psrt_probe_f64(int op, const double* __restrict__ x,
                               const double* __restrict__ y, double* __restrict__ out,
                               unsigned n) {
  const unsigned e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  double r;
  switch (op) {
    case 0: r = __builtin_sqrt(x[e]); break;
    case 1: r = x[e] / y[e]; break;
    case 2: r = x[e] * y[e]; break;
    case 3: r = x[e] + y[e]; break;
    case 4: r = x[e] * y[e] + x[e]; break;  // must NOT contract
    case 6: r = sqrt_f64(x[e]); break;        // the trace kernel's sqrt (fast path + fallback)

    default: r = __builtin_ldexp(x[e], (int)y[e]); break;
  }
  out[e] = r;
}

}  // namespace psrt
