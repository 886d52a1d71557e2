// psrt_kernels.h — launch arguments shared by the kernels and the C ABI host.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace psrt {

#ifndef PSRT_TRACE_BLOCK
#define PSRT_TRACE_BLOCK 512  // 8 waves per workgroup (3 per CU share 160 KB of LDS)
#endif
constexpr int kTraceBlock = PSRT_TRACE_BLOCK;
#ifndef PSRT_WORK_CHUNK
#define PSRT_WORK_CHUNK 1024  // 512 before frame pipelining (C3 pipelined 16.00 -> 15.85 ms)
#endif
constexpr unsigned kWorkChunk = PSRT_WORK_CHUNK;  // largest queue ticket (units); see queue_phases
constexpr unsigned kLinearChunk = 1024;           // queue ticket of the small-scene (linear) path
constexpr int kQueuePhases = 5;        // guided: ticket sizes halve toward the end, >= 64
#ifndef PSRT_QUEUES
#define PSRT_QUEUES 8
#endif
// Queue heads and statistics counters are sharded: blocks b and b + 8 share an
// XCD (round-robin placement), and blocks with label b % kQueues share one
// head / counter set on its own 128-B line. One device-scope head saturates
// near 88 dequeues/us (MI355X_MICROARCH.md, "dequeue"); small tickets (C1,
// small shards) ran into that. Global ticket g = t * kQueues + label, where t
// counts the tickets taken from the label's head; a wave whose head runs past
// the end of the work moves on to the next heads (stealing) before it stops.
constexpr int kQueues = PSRT_QUEUES;
constexpr int kShardStride = 16;       // u64 words between heads / counter sets (128 B)
// Statistics words of a counter set / the render's totals: [0] rays, [1] full
// FP64 sphere tests, [2] FP32 box tests, [3] traced rays, [4] FP32 sphere
// pre-rejects, [5] FP64 root-box tests ([1], [2], [4], [5]: counting variant only)
constexpr int kStatWords = 6;
// Scene data psrt_trace stages in (dynamic) LDS per workgroup: BVH nodes (2
// float4 each, plus the padding node), spheres {c, r*r}, 1/r, leaf slots and
// neighbour records (8 B), FP32 pre-reject spheres and the big-sphere
// indices; byte offsets, 16-B aligned. The host stages them when as
// many workgroups per CU stay resident as without (C3: 573 nodes, 485
// spheres, 41.6 KB; three workgroups).
struct LdsLayout {
  unsigned nodes, sph, leaf, big, bytes;
};
// One 64-B record per sphere (r04): the sphere {c, r*r}, its FP32 pre-reject
// sphere (BvhView::geo32), its neighbour record (BvhView::nb_rec) and 1/r, so
// a sphere's fields share one base register and one index computation.
struct LdsSphere {
  double4 geo;
  float4 g32;
  uint2 nb;
  double inv;
};
static_assert(sizeof(LdsSphere) == 64, "LDS sphere record");
__host__ __device__ inline LdsLayout lds_layout(int n, int n_nodes, int n_leaf, int n_big) {
  auto a16 = [](unsigned x) { return (x + 15u) & ~15u; };
  LdsLayout l;
  l.nodes = 0;                                 // the walk's array at a constant address
  l.sph = 32u * (unsigned)(n_nodes + 1);       // LdsSphere [n]
  l.leaf = l.sph + 64u * (unsigned)n;          // leaf slots [n_leaf]
  l.big = a16(l.leaf + 4u * (unsigned)n_leaf);  // big-sphere indices [n_big]
  l.bytes = a16(l.big + 4u * (unsigned)(n_big > 0 ? n_big : 1));
  return l;
}

// Division of n < 2^32 by an invariant d: q = (t + ((n - t) >> sh1)) >> sh2,
// t = mulhi(m, n) (host: FastDiv::make).
struct FastDiv {
  unsigned m, sh1, sh2, d;
};

// Sample record: t (double) and k (uint16); k = kSampleBlack for a black sample.
constexpr unsigned short kSampleBlack = 0xFFFFu;
constexpr int kSampleKCap = 1100;
constexpr int kReduceBlock = 64;   // psrt_reduce: one wave per 64 pixels
#ifndef PSRT_REDUCE_IN_FLIGHT
#define PSRT_REDUCE_IN_FLIGHT 2
#endif
constexpr unsigned kReduceInFlight = PSRT_REDUCE_IN_FLIGHT;  // psrt_reduce: sample tiles in flight per wave
#ifndef PSRT_REDUCE_TILE
#define PSRT_REDUCE_TILE 32
#endif
constexpr int kReduceTile = PSRT_REDUCE_TILE;  // samples per pixel per LDS tile: 16 or 32
constexpr size_t kSampleBytes = sizeof(double) + sizeof(unsigned short);


// Frames of one multi-frame launch (rt_render_device_frames): the same shard
// and scene, frame f with seed + f; the launch tail is paid once per batch.
constexpr int kMaxFrames = 32;

struct TraceArgs {
  int n;               // spheres (geo: {cx, cy, cz, r*r}, inv_r: 1.0/r)
  double org[3], llc[3], hor[3], ver[3];
  int width, height, max_depth;
  int row_offset, row_stride;
  unsigned pixels;      // rows_owned * width
  int s_begin, s_count; // sample chunk [s_begin, s_begin + s_count)
  int frames;           // frames of this launch, 1..kMaxFrames: unit u = (f * pixels + q) *
                        // s_count + s, frame f's records at [f * pixels * s_count, ...)
  uint64_t total_units; // frames * pixels * s_count  (< 2^32)
  uint64_t seedmix[kMaxFrames];  // splitmix64(seed + f) per frame f
  unsigned long long* work_counter;  // kQueues heads, kShardStride apart (one atomicAdd per ticket)
  // Guided work queue: tickets [ph_first[p], ph_first[p+1]) of phase p cover
  // ph_size[p] units each from unit ph_base[p] on; the last phase is open.
  // Sizes shrink toward the end of the queue, so the last windows are small
  // and the waves finish together (host: queue_phases in psrt_capi.hip).
  uint64_t ph_first[kQueuePhases + 1];
  uint64_t ph_base[kQueuePhases];
  unsigned ph_size[kQueuePhases];
  unsigned long long* ray_counter;  // kQueues sets, kShardStride apart: kStatWords counters
                                    // (rays, tests by kind, traced rays; psrt_reduce sums them)
  unsigned long long* stamps;       // diagnostic build: cycles per section (kSecCount)
  unsigned long long* wave_log;     // diagnostic build: per wave {start, queue empty, exit,
                                    // iterations at queue empty, at exit} (s_memrealtime,
                                    // 100 MHz), or nullptr
  FastDiv div_s, div_w, div_p;      // unit / s_count, q / width, (f * pixels + q) / pixels
  unsigned flush_at;                // per-lane counters flush to the totals at this value
  int tail_prio;                    // raise the issue priority of waves whose queue is empty
  // Drain flag (rt_context_wait_drain): every wave that finds the work queue
  // empty stores drain_epoch here, so another stream can start the next
  // frame's launch as this one's tail begins (nullptr: none)
  unsigned long long* drain_flag;
  unsigned long long drain_epoch;
};

// BVH node as the device reads it (two float4, from psrt_bvh.h BvhNode):
// {lo.x, lo.y, hi.x, hi.y}, {lo.z, hi.z, skip, leaf} (skip / leaf: int bits),
// so the slab test's coordinate pairs are adjacent (packed FP32 FMAs).
struct DevNode {
  float4 xy, z;
};
static_assert(sizeof(DevNode) == 32, "device node layout");

struct BvhView {
  const float4* __restrict__ nodes;      // DevNode as 2 x float4
  const double4* __restrict__ leaf_geo;  // sphere per leaf slot
  const int* __restrict__ leaf_idx;      // original index per leaf slot
  const int* __restrict__ big_idx;       // spheres tested on every ray
  int n_nodes, n_big, n_leaf;
  // first node of a walk: 1 when the root is interior (every parked ray is
  // inside its box, or re-based onto it: testing it is wasted), else 0
  int walk0;
  double r_check;
  // point-location grid (psrt_bvh.h GridHost)
  const int* __restrict__ cell_start;
  const int* __restrict__ cell_items;
  float glo[3], ghi[3], ginv, gmargin;  // FP32 copies (conservative use only)
  int gdims[3];
  int fixpoint;  // end provably trapped paths early (hit_quick; RT_FLAG_NO_FIXPOINT clears it)
  // per-pixel candidate lists for camera rays (psrt_camera_lists), or nullptr:
  // {count | idx0 << 16, idx1 | idx2 << 16, ...}: up to 7 BVH-sphere indices
  // (uint16); count 0xFFFF = overflow (the ray walks the BVH)
  const uint4* __restrict__ plist;
  // neighbour lists (psrt_bvh.h): nb_word[j] = first << 4 | count, -1 = grid
  const int* __restrict__ nb_word;
  const int* __restrict__ nb_items;
  double nb_c2;  // (pad/2)^2: C <= 0 or C^2 <= nb_c2 * r^2 puts o in j's padded ball
  // the grid lists and neighbour lists as inline records (psrt_bvh.h
  // BvhHost::cell_rec / nb_rec, the plist format): psrt_trace's hit_quick
  // reads one record per query instead of an offset pair and the items
  const uint4* __restrict__ cell_rec;  // [2 * ncell]
  const uint2* __restrict__ nb_rec;    // [n]
  // per sphere {fl(cx), fl(cy), fl(cz), R}, R >= |r| + 2^-18 (|c|inf + |r|) +
  // 2^-60 rounded up (+inf beyond 2^40): the FP32 pre-reject (psrt_kernels.hip
  // Pre32) of test_sphere
  const float4* __restrict__ geo32;    // [n]
};

constexpr int kCamTile = 8;         // camera-list tiles are 8 x 8 pixels (one wave)
constexpr int kCamTileCap = 1024;   // tile candidates held in LDS
constexpr int kCamPixelCap = 7;     // candidates per pixel record
constexpr unsigned kCamOverflow = 0xFFFFu;

struct CamListArgs {
  double org[3], llc[3], hor[3], ver[3];
  int width, height, row_offset, row_stride, rows;
  const double4* __restrict__ leaf_geo;  // BVH spheres {cx, cy, cz, r*r} per leaf slot
  const int* __restrict__ leaf_idx;      // original index per leaf slot
  int n_leaf;
  double pad;                            // BVH box padding (absolute)
  uint4* __restrict__ plist;             // [rows * width]
};

struct ReduceArgs {
  const double* samp_t;           // [pixels][s_count] (unit order) sky parameter t (sample_colour)
  const unsigned short* samp_k;   // [pixels][s_count] hits, or kSampleBlack
  unsigned pixels;
  int s_count;
  int first_chunk;
  int spp_total;
  double inv_spp;         // 1.0 / spp_total (psrt_reduce_lean: the division on the host)
  double* accum;          // [pixels][3] (required unless single chunk + rgb only)
  unsigned char* rgb8;    // [pixels][3] or nullptr (last chunk only)
  int fold_stats;         // block 0 folds the counter sets (one reduce per launch: frame 0's)
  // every k < 1000 (max_depth <= 1000): 0.5^k is one ldexp, no halving loop,
  // and a sample's colour is formed without branches (psrt_reduce)
  int fast_k;
  // psrt_reduce over the frames of a multi-frame launch in ONE launch (r04):
  // blockIdx.y = frame f, whose records start f * frame_units into samp_t /
  // samp_k and whose sums / bytes go to accum + f * accum_stride / rgb8 +
  // f * rgb8_stride (the caller's frames evenly strided; plain offsets: an
  // array of pointers in the arguments, indexed by f, put them in scratch)
  size_t frame_units;
  size_t accum_stride;  // doubles
  size_t rgb8_stride;   // bytes
  // Row pitches of the outputs (rt_context_set_row_pitch), 0 = packed rows:
  // pixel q = row * width + i of the shard at accum + row * accum_pitch + 3 i
  // (doubles) and rgb8 + row * rgb8_pitch + 3 i (bytes), so G shards can write
  // their interleaved rows straight into one frame
  size_t accum_pitch, rgb8_pitch;
  unsigned width;
  // Statistics and queue state of the trace launch before this reduce
  // (block 0 only): the counter sets are added into totals (reset on the first
  // chunk), then the sets and the queue heads are zeroed for the next launch;
  // the last chunk also writes totals to host_stats (pinned host memory).
  unsigned long long* heads;       // TraceArgs::work_counter (kQueues heads)
  unsigned long long* sets;        // TraceArgs::ray_counter (kQueues sets)
  unsigned long long* totals;      // [kStatWords], device
  unsigned long long* host_stats;  // [kStatWords], or nullptr
};

// ---- material integrator (psrt_mat.hip) ----
// One material per sphere (rt_material, fuzz clamped to <= 1 by the host).
struct DevMaterial {
  double albedo[3];
  double fuzz;
  double ir;
  int kind;  // RT_MAT_*
  int pad_;
};
static_assert(sizeof(DevMaterial) == 48, "device material layout");
#ifndef PSRT_MAT_BLOCK
#define PSRT_MAT_BLOCK 512  // 8 waves: two workgroups per CU share 160 KB of LDS
#endif
constexpr int kMatBlock = PSRT_MAT_BLOCK;
#ifndef PSRT_MAT_WAVES
// waves per SIMD asked of the register allocator: 4 (up to 128 VGPRs) —
// LDS already holds the kernel to two 512-thread workgroups (4 waves per
// SIMD); 5 (96 VGPRs) cost 3% (r04, profiles/r04_matlist)
#define PSRT_MAT_WAVES 4
#endif
constexpr int kMatWaves = PSRT_MAT_WAVES;
constexpr unsigned kMatChunk = 256;  // units per queue ticket
constexpr int kMatMaxDepth = 4096;   // path scratch rows (max_depth bound of RT_FLAG_MATERIALS)
// Sample record of the material path: the sample's colour, 3 doubles, in unit
// order (unit u = (f * pixels + q) * s_count + s, as TraceArgs).
constexpr size_t kMatSampleBytes = 3 * sizeof(double);

struct MatArgs {
  int n;
  double org[3], llc[3], hor[3], ver[3];  // focus-plane basis (camera get_ray)
  double lu[3], lv[3], lens_radius;       // thin lens: offset = lu rd.x + lv rd.y
  int width, height, max_depth;
  int row_offset, row_stride;
  unsigned pixels;
  int s_begin, s_count, frames;
  uint64_t total_units;  // frames * pixels * s_count (< 2^32)
  uint64_t seedmix[kMaxFrames];
  FastDiv div_s, div_w, div_p;
  unsigned long long* work_counter;  // kQueues heads, kShardStride apart
  unsigned long long* ray_counter;   // kQueues counter sets (as TraceArgs)
  const DevMaterial* __restrict__ mats;
  // per resident lane, the attenuating (non-dielectric) hits of its path:
  // path[k * path_stride + lane slot], k < max_depth
  int* __restrict__ path;
  unsigned path_stride;
  unsigned batch;  // parked lanes that trigger a batched BVH walk
  // per-pixel candidate lists of the camera rays through the lens
  // (psrt_mat_camera_lists; CamListArgs format), or nullptr
  const uint4* __restrict__ plist;
};

// Camera-ray candidate lists for the thin lens (psrt_mat_camera_lists):
// every ray of pixel (i, j) starts on the lens disk (radius lens_radius about
// the origin) and passes through the pixel's patch of the focus plane.
struct MatCamListArgs {
  double org[3], llc[3], hor[3], ver[3];
  double lens_radius;
  int width, height, row_offset, row_stride, rows;
  const double4* __restrict__ leaf_geo;  // BVH spheres {cx, cy, cz, r*r} per leaf slot
  const int* __restrict__ leaf_idx;      // original index per leaf slot
  int n_leaf;
  double pad;                            // BVH box padding (absolute)
  uint4* __restrict__ plist;             // [rows * width]
};

// psrt_trace_mat<true, true> stages the scene in dynamic LDS: BVH nodes (2
// float4 each, plus the padding node), leaf spheres, spheres {c, r*r} and
// 1/r by index, materials {albedo, fuzz or ir} and kinds by index, leaf
// indices, big-sphere indices; byte offsets, 16-B aligned (book scene: 487
// spheres, 71 KB; two 512-thread workgroups per CU)
struct MatLdsLayout {
  unsigned nodes, leaf_geo, geo, mat, inv, leaf_idx, kind, big, bytes;
};
__host__ __device__ inline MatLdsLayout mat_lds_layout(int n, int n_nodes, int n_leaf, int n_big) {
  auto a16 = [](unsigned x) { return (x + 15u) & ~15u; };
  MatLdsLayout l;
  l.nodes = 0;
  l.leaf_geo = 32u * (unsigned)(n_nodes + 1);
  l.geo = l.leaf_geo + 32u * (unsigned)n_leaf;
  l.mat = l.geo + 32u * (unsigned)n;
  l.inv = l.mat + 32u * (unsigned)n;
  l.leaf_idx = a16(l.inv + 8u * (unsigned)n);
  l.kind = a16(l.leaf_idx + 4u * (unsigned)n_leaf);
  l.big = a16(l.kind + 4u * (unsigned)n);
  l.bytes = a16(l.big + 4u * (unsigned)(n_big > 0 ? n_big : 1));
  return l;
}

template <bool kBVH, bool kLds, bool kCount>
__global__ void psrt_trace_mat(const double4* __restrict__ geo, const double* __restrict__ inv_r,
                               double* __restrict__ rgb, MatArgs a, BvhView bv);
// psrt_reduce over colour records: samp_t holds [pixels][s_count][3] doubles
__global__ void psrt_reduce_rgb(ReduceArgs a);
__global__ void psrt_mat_camera_lists(MatCamListArgs a);

template <bool kBVH, bool kStamps, bool kLds, bool kCount>
__global__ void psrt_trace(const double4* __restrict__ geo, const double* __restrict__ inv_r,
                           double* __restrict__ samples, TraceArgs a, BvhView bv);
__global__ void psrt_reduce(ReduceArgs a);
// psrt_reduce in 16 SGPRs, 32 VGPRs and no LDS: fits beside a resident
// psrt_trace (Tuning reduce_lean; frames in flight); no statistics fold
__global__ void psrt_reduce_lean(ReduceArgs a);
// psrt_reduce's statistics fold alone, in psrt_reduce_lean's register budget
__global__ void psrt_fold_stats(ReduceArgs a);
__global__ void psrt_camera_lists(CamListArgs a);
__global__ void psrt_quantize(const double* __restrict__ accum, unsigned char* __restrict__ rgb8,
                              unsigned n, int spp);
__global__ void psrt_probe_hit(const double4* __restrict__ geo, const double* __restrict__ inv_r,
                               int n, const double* __restrict__ rays, const int* __restrict__ hints,
                               double* __restrict__ out, unsigned count, BvhView bv, int use_bvh);
__global__ void psrt_probe_f64(int op, const double* __restrict__ x, const double* __restrict__ y,
                               double* __restrict__ out, unsigned n);

}  // namespace psrt
