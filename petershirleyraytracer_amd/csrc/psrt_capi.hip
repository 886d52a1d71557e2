// psrt_capi.hip — the C ABI of include/rt.h on HIP.
//
// Replaces the reference's pixel loop (main.cc:72-88) for a shard of rows:
// the scene arrives flattened (rt_sphere[], rt_camera), device buffers are
// owned by an rt_context, and one render enqueues, per sample chunk, one
// psrt_trace megakernel launch and one psrt_reduce launch on a HIP stream.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <mutex>
#include <string>
#include <type_traits>
#include <vector>

#include "../../include/rt.h"
#include "psrt_bvh.h"
#include "psrt_error.h"
#include "psrt_kernels.h"

namespace {
thread_local std::string g_err;
}  // namespace

namespace psrt {
int set_error(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  std::vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}
}  // namespace psrt

namespace {

using psrt::set_error;

#define HIP_TRY(expr)                                                                  \
  do {                                                                                 \
    hipError_t e_ = (expr);                                                            \
    if (e_ != hipSuccess)                                                              \
      return set_error(e_ == hipErrorOutOfMemory ? RT_E_NOMEM : RT_E_HIP, "%s: %s (%s:%d)", \
                  #expr, hipGetErrorString(e_), __FILE__, __LINE__);                   \
  } while (0)

uint64_t splitmix64_host(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ULL;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

// Magic numbers for n / d, n < 2^32 (psrt_kernels.h FastDiv): l = ceil(log2 d),
// m = floor(2^32 (2^l - d) / d) + 1.
psrt::FastDiv fast_div_make(unsigned d) {
  unsigned l = 0;
  while (l < 32 && (1ull << l) < d) ++l;
  psrt::FastDiv f;
  f.m = (unsigned)(((1ull << 32) * ((1ull << l) - d)) / d + 1);
  f.sh1 = l ? 1u : 0u;
  f.sh2 = l ? l - 1 : 0u;
  f.d = d;
  return f;
}

// d_counters layout (words): [1, 1 + kStatWords) totals (psrt_reduce), [8, 128) stamps
constexpr size_t kTotals = 1;
constexpr size_t kHeads = 128;
constexpr size_t kSets = kHeads + (size_t)psrt::kQueues * psrt::kShardStride;
constexpr size_t kCounterWords = kSets + (size_t)psrt::kQueues * psrt::kShardStride;

// HBM left to the GPU's other users when the sample buffer is sized to the
// free memory (rt_render_device)
constexpr size_t kHbmReserve = (size_t)256 << 20;

}  // namespace

namespace psrt {
// Tuning knobs (rt_context_set_tuning; measurement and tests only). The
// render path reads no environment variable: a context copies the process
// defaults at creation, the one-shot entries' default contexts at each call.
// Every knob keeps the output bit-identical.
struct Tuning {
  // sample-record buffer cap: 48 GiB of the 288 GB HBM holds C4 on one GPU
  // (41 GB of records) in one chunk, C5 (96 GB) in 3; fewer chunks, fewer
  // launch tails (measured: C4 564 -> 561 ms, C5 1312 -> 1306 ms against 16 GiB)
  double sample_buf_mb = 49152;
  double queue_k = 2, queue_d = 2;  // guided work queue shape (queue_phases)
  double linear_chunk = 0;          // small-scene queue ticket (0: kLinearChunk)
  double no_camlist = 0, no_neighbors = 0, no_fixpoint = 0, no_lds = 0;
  double blocks_per_cu = 0;  // cap on resident trace workgroups per CU (0: occupancy max)
  double mat_lds = -1;       // material kernel's scene in LDS: -1 auto, 0 off, 1 on
  double mat_batch = 48;     // parked lanes per batched material walk (40-56 best, profiles/r03_mat)
  double flush_at = 0;       // per-lane counter flush threshold (0: computed; tests force it low)
  double stamps = 0;         // diagnostic kernel variant (section clocks, utilisation probes)
  double scene_rebuild = 0;  // rebuild the culling structures for an unchanged scene
  double big_ratio = 0;      // radius ratio of the big-sphere class (0: psrt_bvh's default)
  double reduce_lean = 0;    // psrt_reduce_lean (fits beside a resident trace: frames in flight)
};
}  // namespace psrt

namespace {

// Each knob's valid range: every later use casts the value to an integer type
// or multiplies it into a size, so rt_context_set_tuning rejects anything
// outside [lo, hi] (RT_E_INVALID) instead of letting a cast wrap.
struct TuningKey {
  const char* name;
  double psrt::Tuning::*field;
  double lo, hi;
};
const TuningKey kTuningKeys[] = {
    {"sample_buf_mb", &psrt::Tuning::sample_buf_mb, 1, 1 << 22},  // 1 MiB .. 4 TiB
    {"queue_k", &psrt::Tuning::queue_k, 0, 64},
    {"queue_d", &psrt::Tuning::queue_d, 0.125, 64},
    {"linear_chunk", &psrt::Tuning::linear_chunk, 0, 1 << 20},
    {"no_camlist", &psrt::Tuning::no_camlist, 0, 1},
    {"no_neighbors", &psrt::Tuning::no_neighbors, 0, 1},
    {"no_fixpoint", &psrt::Tuning::no_fixpoint, 0, 1},
    {"no_lds", &psrt::Tuning::no_lds, 0, 1},
    {"blocks_per_cu", &psrt::Tuning::blocks_per_cu, 0, 64},
    {"mat_lds", &psrt::Tuning::mat_lds, -1, 1},
    {"mat_batch", &psrt::Tuning::mat_batch, 1, 64},
    {"flush_at", &psrt::Tuning::flush_at, 0, 4294967295.0},
    {"stamps", &psrt::Tuning::stamps, 0, 1},
    {"scene_rebuild", &psrt::Tuning::scene_rebuild, 0, 1},
    {"big_ratio", &psrt::Tuning::big_ratio, 0, 1e300},
    {"reduce_lean", &psrt::Tuning::reduce_lean, 0, 1},
};
std::mutex g_tuning_mu;
psrt::Tuning g_tuning;  // the process defaults (rt_context_set_tuning(NULL, ...))

psrt::Tuning tuning_defaults() {
  std::lock_guard<std::mutex> lk(g_tuning_mu);
  return g_tuning;
}

size_t sample_buffer_cap_bytes(const psrt::Tuning& t) {
  const double mb = t.sample_buf_mb >= 1 ? t.sample_buf_mb : 1;
  return (size_t)mb << 20;
}

}  // namespace

struct rt_context {
  int device = 0;
  int cus = 0;
  int grid = 0;       // resident blocks of psrt_trace<false>
  int grid_bvh = 0;   // resident blocks of psrt_trace<true>
  unsigned lds_max = 0;  // largest dynamic LDS that keeps grid_bvh resident (staged scenes)
  // exact-culling structure (psrt_bvh.h)
  bool bvh = false;
  float4* d_nodes = nullptr;
  double4* d_leaf_geo = nullptr;
  int* d_leaf_idx = nullptr;
  int* d_big = nullptr;
  int* d_cell_start = nullptr;
  int* d_cell_items = nullptr;
  int* d_nb_word = nullptr;
  int* d_nb_items = nullptr;
  uint4* d_cell_rec = nullptr;  // grid lists as inline records (BvhHost::cell_rec)
  uint2* d_nb_rec = nullptr;    // neighbour lists as inline records (BvhHost::nb_rec)
  std::vector<rt_sphere> scene;   // the scene the structures were built for
  double built_big_ratio = 0;     // Tuning::big_ratio the structures were built with
  psrt::GridHost pgrid;  // point-location grid (host copy of the geometry)
  double pad = 0.0;
  int n_nodes = 0, n_big = 0, n_leaf = 0;
  int walk0 = 0;  // BvhView::walk0
  double r_check = 0.0;
  hipStream_t stream = nullptr;
  double4* d_geo = nullptr;
  double* d_inv_r = nullptr;
  float4* d_geo32 = nullptr;  // the FP32 pre-reject's spheres (psrt_kernels.h BvhView::geo32)
  int n = -1;
  int n_cap = 0;
  rt_camera cam{};
  double* d_samples = nullptr;
  size_t samples_cap = 0;  // doubles
  double* d_accum_tmp = nullptr;
  size_t accum_tmp_cap = 0;  // doubles
  // the material integrator's camera-ray lists through the lens
  // (psrt_mat_camera_lists), cached per (materials / lens camera, W, H,
  // row_offset, row_stride)
  uint4* d_mat_plist = nullptr;
  size_t mat_plist_cap = 0;  // records
  bool mat_plist_valid = false;
  int mat_plist_key[4] = {0, 0, 0, 0};
  uint4* d_plist = nullptr;  // camera-ray candidate lists, one uint4 per owned pixel
  size_t plist_cap = 0;      // records
  // The lists depend only on the scene, camera, frame size and shard: they
  // are built once per (set_scene, W, H, row_offset, row_stride) and reused.
  bool plist_valid = false;
  int plist_key[4] = {0, 0, 0, 0};
  hipEvent_t ev_plist = nullptr;  // after the lists' build (other streams wait on it)
  hipEvent_t ev_mat_plist = nullptr;  // the same for the material lists
  unsigned long long* d_wave_log = nullptr;  // diagnostic (PSRT_STAMPS): per-wave timeline
  size_t wave_log_cap = 0, wave_log_used = 0;
  // [8, 128) diagnostic stamps; queue heads at kHeads, statistics counter sets
  // (rays, sphere tests, box tests, traced rays) at kSets, kShardStride apart
  unsigned long long* d_counters = nullptr;
  // The render's statistics, written by its last psrt_reduce straight into
  // pinned host memory: reading them back needs no copy kernel, which (like
  // any kernel) would wait for a free CU slot behind the next frame's
  // persistent trace launch
  unsigned long long* h_stats = nullptr;  // [kStatWords] host pointer
  unsigned long long* d_stats = nullptr;  // the same memory, device pointer
  std::vector<hipEvent_t> ev;  // pairs around each trace launch
  int ev_used = 0;
  hipEvent_t ev_all0 = nullptr, ev_all1 = nullptr;
  hipStream_t last_stream = nullptr;  // stream of the last render (stats readback)
  // A render was enqueued and ev_all1 marks its end. The device buffers above
  // are shared by every render of the context, whatever its stream: a render
  // on another stream waits for ev_all1 on the device, and host-side writes
  // (set_scene, reallocation) wait for it on the host (quiesce).
  bool in_flight = false;
  // a render failed after its first trace launch: queue heads / counter sets
  // may be non-zero until the next render re-zeroes them (stream-ordered)
  bool dirty = false;
  // material integrator (rt_context_set_materials)
  int grid_mat = 0, grid_mat_bvh = 0;  // resident blocks of psrt_trace_mat<false / true>
  bool has_mats = false;               // materials set for the current scene
  psrt::DevMaterial* d_mats = nullptr;
  int mats_cap = 0;
  rt_camera_lens lcam{};
  int* d_path = nullptr;  // per resident lane, its path's attenuating hits
  size_t path_cap = 0;    // ints
  rt_stats last{};
  int n_last = 0;
  bool last_mat = false;  // the last render used RT_FLAG_MATERIALS (no stamps to read)
  bool failed = false;    // the last render failed part-way (its timings are not reported)
  int fail_after = -1;    // rt_debug_fail_after_trace: the next render fails after this chunk
  psrt::Tuning tune;      // rt_context_set_tuning
  // rt_context_set_row_pitch: rows of the outputs this far apart (0: packed)
  size_t accum_pitch = 0;  // doubles
  size_t rgb8_pitch = 0;   // bytes
  bool last_stamps = false;  // the last render ran the diagnostic variant (tune.stamps)
  // Drain flag (rt_context_wait_drain): HSA signal memory that each trace
  // launch's waves set to its epoch once its work queue is empty; epochs count
  // the context's enqueued trace launches (never reset, so a late wait holds)
  unsigned long long* d_drain = nullptr;
  unsigned long long drain_epoch = 0;
  // psrt_reduce_lean fits beside a resident trace only within 32 VGPRs (and
  // 16 SGPRs: tests/test_abi.py reads the code object's counts)
  bool lean_ok = false;
};

namespace {

int ensure_events(rt_context* c, int pairs) {
  while ((int)c->ev.size() < 2 * pairs) {
    hipEvent_t e;
    HIP_TRY(hipEventCreate(&e));
    c->ev.push_back(e);
  }
  return RT_OK;
}

// Host wait for the context's last enqueued render (any stream): before the
// host writes or frees a buffer that render may still read.
int quiesce(rt_context* c) {
  if (c->stream) HIP_TRY(hipStreamSynchronize(c->stream));
  if (c->in_flight) HIP_TRY(hipEventSynchronize(c->ev_all1));
  return RT_OK;
}

int ensure_buf(rt_context* c, double** p, size_t* cap, size_t need) {
  if (*cap >= need && *p) return RT_OK;
  const int rc = quiesce(c);
  if (rc) return rc;
  if (*p) (void)hipFree(*p);
  *p = nullptr;
  *cap = 0;
  HIP_TRY(hipMalloc(p, need * sizeof(double)));
  *cap = need;
  return RT_OK;
}

// Scratch device allocation of a debug entry: freed on every return path,
// after the context's stream (which may still read it) has drained.
struct ScratchBuf {
  void* p = nullptr;
  hipStream_t st = nullptr;
  explicit ScratchBuf(hipStream_t s) : st(s) {}
  ScratchBuf(const ScratchBuf&) = delete;
  ScratchBuf& operator=(const ScratchBuf&) = delete;
  ~ScratchBuf() {
    if (!p) return;
    (void)hipStreamSynchronize(st);
    (void)hipFree(p);
  }
  template <class T>
  T* as() const { return static_cast<T*>(p); }
};

std::mutex g_default_mu;
rt_context* g_default[64] = {};
// One-shot entries (rt_render, rt_debug_*) share their device's default
// context: each holds that device's lock for the whole call.
std::mutex g_device_mu[64];

// RT_DEVICE (include/rt.h: the one-shot entries' device), read once
int default_device() {
  static const int dev = [] {
    const char* e = std::getenv("RT_DEVICE");
    return e ? std::atoi(e) : 0;
  }();
  return dev;
}

}  // namespace

extern "C" {

const char* rt_last_error(void) { return g_err.c_str(); }
int rt_abi_version(void) { return RT_ABI_VERSION; }

const char* rt_build_info(void) {
#define PSRT_STR2(x) #x
#define PSRT_STR(x) PSRT_STR2(x)
  return "psrt gfx950 megakernel (fp64 exact, -ffp-contract=off); trace block " PSRT_STR(
      PSRT_TRACE_BLOCK) ", work chunk " PSRT_STR(PSRT_WORK_CHUNK);
}

int rt_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int rt_rows_owned(int height, int row_offset, int row_stride) {
  if (height <= 0 || row_stride <= 0 || row_offset < 0 || row_offset >= height) return 0;
  return (height - 1 - row_offset) / row_stride + 1;
}

int rt_context_create(int device, rt_context** out) {
  if (!out) return set_error(RT_E_INVALID, "rt_context_create: out is NULL");
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
    return set_error(RT_E_NODEVICE, "rt_context_create: no HIP device visible");
  if (device < 0 || device >= ndev)
    return set_error(RT_E_INVALID, "rt_context_create: device %d out of range [0,%d)", device, ndev);
  HIP_TRY(hipSetDevice(device));
  rt_context* c = new rt_context();
  c->device = device;
  c->tune = tuning_defaults();
  hipDeviceProp_t prop;
  HIP_TRY(hipGetDeviceProperties(&prop, device));
  c->cus = prop.multiProcessorCount;
  int per_cu = 0;
  HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, psrt::psrt_trace<false, false, false, false>,
                                                        psrt::kTraceBlock, 0));
  c->grid = c->cus * (per_cu < 1 ? 1 : per_cu);
  HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, psrt::psrt_trace<true, false, false, false>,
                                                        psrt::kTraceBlock, 0));
  c->grid_bvh = c->cus * (per_cu < 1 ? 1 : per_cu);
  // the staged-scene variant keeps that residency up to lds_max bytes of
  // dynamic LDS (largest multiple of 256 B the occupancy query accepts)
  for (unsigned b = 65536; b >= 256; b -= 256) {
    int pc = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&pc, psrt::psrt_trace<true, false, true, false>,
                                                     psrt::kTraceBlock, b) == hipSuccess &&
        pc >= per_cu) {
      c->lds_max = b;
      break;
    }
  }
  HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, psrt::psrt_trace_mat<false, false, false>,
                                                        psrt::kMatBlock, 0));
  c->grid_mat = c->cus * (per_cu < 1 ? 1 : per_cu);
  HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, psrt::psrt_trace_mat<true, false, false>,
                                                        psrt::kMatBlock, 0));
  c->grid_mat_bvh = c->cus * (per_cu < 1 ? 1 : per_cu);
  {
    hipFuncAttributes fa{};
    HIP_TRY(hipFuncGetAttributes(&fa, (const void*)psrt::psrt_reduce_lean));
    c->lean_ok = fa.numRegs <= 32 && fa.sharedSizeBytes == 0;
    HIP_TRY(hipFuncGetAttributes(&fa, (const void*)psrt::psrt_fold_stats));
    c->lean_ok = c->lean_ok && fa.numRegs <= 32 && fa.sharedSizeBytes == 0;
  }
  HIP_TRY(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
  HIP_TRY(hipMalloc(&c->d_counters, kCounterWords * sizeof(unsigned long long)));
  // zeroed once: psrt_reduce leaves the queue heads and counter sets at zero
  HIP_TRY(hipMemsetAsync(c->d_counters, 0, kCounterWords * sizeof(unsigned long long), c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  HIP_TRY(hipHostMalloc((void**)&c->h_stats, psrt::kStatWords * sizeof(unsigned long long),
                        hipHostMallocMapped | hipHostMallocCoherent));
  HIP_TRY(hipHostGetDevicePointer((void**)&c->d_stats, c->h_stats, 0));
  std::fill(c->h_stats, c->h_stats + psrt::kStatWords, 0ull);
  HIP_TRY(hipEventCreate(&c->ev_all0));
  HIP_TRY(hipEventCreate(&c->ev_all1));
  HIP_TRY(hipEventCreateWithFlags(&c->ev_plist, hipEventDisableTiming));
  HIP_TRY(hipEventCreateWithFlags(&c->ev_mat_plist, hipEventDisableTiming));
  // the drain flag (optional: without it rt_context_wait_drain reports RT_E_HIP)
  if (hipExtMallocWithFlags((void**)&c->d_drain, sizeof(unsigned long long),
                            hipMallocSignalMemory) != hipSuccess) {
    (void)hipGetLastError();
    c->d_drain = nullptr;
  } else {
    HIP_TRY(hipStreamWriteValue64(c->stream, c->d_drain, 0, 0));
    HIP_TRY(hipStreamSynchronize(c->stream));
  }
  *out = c;
  return RT_OK;
}

int rt_context_destroy(rt_context* c) {
  if (!c) return RT_OK;
  (void)hipSetDevice(c->device);
  (void)quiesce(c);
  if (c->h_stats) (void)hipHostFree(c->h_stats);
  (void)hipFree(c->d_geo);
  (void)hipFree(c->d_inv_r);
  (void)hipFree(c->d_geo32);
  (void)hipFree(c->d_samples);
  (void)hipFree(c->d_accum_tmp);
  (void)hipFree(c->d_plist);
  (void)hipFree(c->d_mat_plist);
  (void)hipFree(c->d_wave_log);
  (void)hipFree(c->d_counters);
  if (c->d_drain) (void)hipFree(c->d_drain);
  (void)hipFree(c->d_nodes);
  (void)hipFree(c->d_leaf_geo);
  (void)hipFree(c->d_leaf_idx);
  (void)hipFree(c->d_big);
  (void)hipFree(c->d_cell_start);
  (void)hipFree(c->d_cell_items);
  (void)hipFree(c->d_nb_word);
  (void)hipFree(c->d_nb_items);
  (void)hipFree(c->d_cell_rec);
  (void)hipFree(c->d_nb_rec);
  (void)hipFree(c->d_mats);
  (void)hipFree(c->d_path);
  for (auto e : c->ev) (void)hipEventDestroy(e);
  if (c->ev_all0) (void)hipEventDestroy(c->ev_all0);
  if (c->ev_all1) (void)hipEventDestroy(c->ev_all1);
  if (c->ev_plist) (void)hipEventDestroy(c->ev_plist);
  if (c->ev_mat_plist) (void)hipEventDestroy(c->ev_mat_plist);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
  return RT_OK;
}

// The FP32 pre-reject's sphere (psrt_kernels.hip test_sphere, Pre32): the
// centre rounded to nearest and R = |r| + 2^-18 (|c|inf + |r|) + 2^-60
// rounded up to FP32; +inf (never rejected) beyond 2^40 or for non-finite input.
static float4 pre32_sphere(const rt_sphere& s) {
  const double ar = std::fabs(s.r);
  const double cm = std::max(std::fabs(s.cx), std::max(std::fabs(s.cy), std::fabs(s.cz)));
  float R = std::numeric_limits<float>::infinity();
  if (cm + ar <= 0x1p40) {  // false for NaN / inf
    // the floor 2^-60 keeps T*T >= 2^-120 a normal float, so its relative
    // error bound holds at any scene scale (tests/host/pre32_check.c)
    const double Rd = ar * (1.0 + 0x1p-18) + 0x1p-18 * cm + 0x1p-60;
    R = (float)Rd;
    if ((double)R < Rd) R = std::nextafter(R, std::numeric_limits<float>::infinity());
  }
  return make_float4((float)s.cx, (float)s.cy, (float)s.cz, R);
}

int rt_context_set_scene(rt_context* c, const rt_sphere* sph, int n, const rt_camera* cam) {
  if (!c || !cam || n < 0 || (n > 0 && !sph))
    return set_error(RT_E_INVALID, "rt_context_set_scene: bad arguments");
  HIP_TRY(hipSetDevice(c->device));
  {  // the last render may run on any stream and still read geo / plist / BVH
    const int rc = quiesce(c);
    if (rc) return rc;
  }
  // The same spheres as the last scene (bit for bit): keep the geometry and
  // the culling structures, only the camera changes (its lists are rebuilt).
  if (n == c->n && n > 0 && (size_t)n == c->scene.size() &&
      std::memcmp(c->scene.data(), sph, (size_t)n * sizeof(rt_sphere)) == 0 &&
      !c->tune.scene_rebuild && c->tune.big_ratio == c->built_big_ratio) {
    c->cam = *cam;
    c->plist_valid = false;
    return RT_OK;
  }
  c->scene.clear();  // set again once every structure is built
  c->has_mats = false;  // materials belong to the scene they were set for
  c->mat_plist_valid = false;
  const int cap = n > 0 ? n : 1;
  if (cap > c->n_cap) {
    (void)hipFree(c->d_geo);
    (void)hipFree(c->d_inv_r);
    (void)hipFree(c->d_geo32);
    c->d_geo = nullptr;
    c->d_inv_r = nullptr;
    c->d_geo32 = nullptr;
    c->n_cap = 0;
    HIP_TRY(hipMalloc(&c->d_geo, cap * sizeof(double4)));
    HIP_TRY(hipMalloc(&c->d_inv_r, cap * sizeof(double)));
    HIP_TRY(hipMalloc(&c->d_geo32, cap * sizeof(float4)));
    c->n_cap = cap;
  }
  // uploads on the context's (non-blocking) stream; synchronised below
  auto up = [c](void* dst, const void* src, size_t bytes) {
    return hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, c->stream);
  };
  // sphere.cc:11 radius*radius and vec3.h:151-154 1/t, each the same IEEE
  // product/quotient the reference forms per call.
  std::vector<double4> geo(cap);
  std::vector<double> inv(cap);
  std::vector<float4> g32(cap);
  for (int k = 0; k < n; ++k) {
    geo[k] = make_double4(sph[k].cx, sph[k].cy, sph[k].cz, sph[k].r * sph[k].r);
    inv[k] = 1 / sph[k].r;
    g32[k] = pre32_sphere(sph[k]);
  }
  if (n > 0) {
    HIP_TRY(up(c->d_geo, geo.data(), n * sizeof(double4)));
    HIP_TRY(up(c->d_inv_r, inv.data(), n * sizeof(double)));
    HIP_TRY(up(c->d_geo32, g32.data(), n * sizeof(float4)));
  }
  c->n = n;
  c->cam = *cam;
  c->plist_valid = false;
  // exact culling structure
  const psrt::BvhHost b = psrt::build_bvh(sph, n, c->tune.big_ratio);
  (void)hipFree(c->d_nodes);
  (void)hipFree(c->d_leaf_geo);
  (void)hipFree(c->d_leaf_idx);
  (void)hipFree(c->d_big);
  (void)hipFree(c->d_cell_start);
  (void)hipFree(c->d_cell_items);
  (void)hipFree(c->d_nb_word);
  (void)hipFree(c->d_nb_items);
  (void)hipFree(c->d_cell_rec);
  (void)hipFree(c->d_nb_rec);
  c->d_nodes = nullptr, c->d_leaf_geo = nullptr, c->d_leaf_idx = nullptr, c->d_big = nullptr;
  c->d_cell_start = nullptr, c->d_cell_items = nullptr;
  c->d_nb_word = nullptr, c->d_nb_items = nullptr;
  c->d_cell_rec = nullptr, c->d_nb_rec = nullptr;
  c->bvh = b.enabled;
  c->n_nodes = c->n_big = c->n_leaf = 0;
  c->walk0 = 0;
  if (b.enabled) {
    c->n_nodes = (int)b.nodes.size() - 1;  // the walk's node count (excl. padding)
    c->n_big = (int)b.big_idx.size();
    c->n_leaf = (int)b.leaf_idx.size();
    c->walk0 = (c->n_nodes > 1 && b.nodes[0].leaf < 0) ? 1 : 0;
    c->r_check = b.r_check;
    std::vector<double4> lg(c->n_leaf);
    for (int k = 0; k < c->n_leaf; ++k) lg[k] = geo[b.leaf_idx[k]];
    HIP_TRY(hipMalloc(&c->d_nodes, b.nodes.size() * sizeof(psrt::DevNode)));
    HIP_TRY(hipMalloc(&c->d_leaf_geo, (size_t)c->n_leaf * sizeof(double4)));
    HIP_TRY(hipMalloc(&c->d_leaf_idx, (size_t)c->n_leaf * sizeof(int)));
    HIP_TRY(hipMalloc(&c->d_big, (size_t)(c->n_big > 0 ? c->n_big : 1) * sizeof(int)));
    std::vector<psrt::DevNode> dn(b.nodes.size());
    for (size_t k = 0; k < dn.size(); ++k) {
      const psrt::BvhNode& nd = b.nodes[k];
      float sk, lf;
      std::memcpy(&sk, &nd.skip, 4);
      std::memcpy(&lf, &nd.leaf, 4);
      dn[k].xy = make_float4(nd.lo[0], nd.lo[1], nd.hi[0], nd.hi[1]);
      dn[k].z = make_float4(nd.lo[2], nd.hi[2], sk, lf);
    }
    HIP_TRY(up(c->d_nodes, dn.data(), dn.size() * sizeof(psrt::DevNode)));
    HIP_TRY(up(c->d_leaf_geo, lg.data(), lg.size() * sizeof(double4)));
    HIP_TRY(up(c->d_leaf_idx, b.leaf_idx.data(), b.leaf_idx.size() * sizeof(int)));
    if (c->n_big > 0)
      HIP_TRY(up(c->d_big, b.big_idx.data(), b.big_idx.size() * sizeof(int)));
    c->pgrid = b.grid;
    c->pad = b.pad;
    const size_t ns = b.grid.start.size(), ni = std::max<size_t>(1, b.grid.items.size());
    HIP_TRY(hipMalloc(&c->d_cell_start, ns * sizeof(int)));
    HIP_TRY(hipMalloc(&c->d_cell_items, ni * sizeof(int)));
    HIP_TRY(up(c->d_cell_start, b.grid.start.data(), ns * sizeof(int)));
    if (!b.grid.items.empty())
      HIP_TRY(up(c->d_cell_items, b.grid.items.data(), b.grid.items.size() * sizeof(int)));
    const size_t nw = b.nb_word.size(), nn = std::max<size_t>(1, b.nb_items.size());
    HIP_TRY(hipMalloc(&c->d_nb_word, std::max<size_t>(1, nw) * sizeof(int)));
    HIP_TRY(hipMalloc(&c->d_nb_items, nn * sizeof(int)));
    if (nw) HIP_TRY(up(c->d_nb_word, b.nb_word.data(), nw * sizeof(int)));
    if (!b.nb_items.empty())
      HIP_TRY(up(c->d_nb_items, b.nb_items.data(), b.nb_items.size() * sizeof(int)));
    HIP_TRY(hipMalloc(&c->d_cell_rec, std::max<size_t>(4, b.cell_rec.size()) * sizeof(uint32_t)));
    HIP_TRY(hipMalloc(&c->d_nb_rec, std::max<size_t>(2, b.nb_rec.size()) * sizeof(uint32_t)));
    if (!b.cell_rec.empty())
      HIP_TRY(up(c->d_cell_rec, b.cell_rec.data(), b.cell_rec.size() * sizeof(uint32_t)));
    if (!b.nb_rec.empty())
      HIP_TRY(up(c->d_nb_rec, b.nb_rec.data(), b.nb_rec.size() * sizeof(uint32_t)));
    // the uploads above read host vectors of this block: wait for them here
    HIP_TRY(hipStreamSynchronize(c->stream));
  }
  // scene uploads run on the context's (non-blocking) stream; renders on it
  // are ordered after them, and returning only once they are done orders
  // renders on any other stream too
  HIP_TRY(hipStreamSynchronize(c->stream));
  c->scene.assign(sph, sph + n);
  c->built_big_ratio = c->tune.big_ratio;
  return RT_OK;
}

static psrt::BvhView bvh_view(const rt_context* c) {
  psrt::BvhView v{};
  v.geo32 = c->d_geo32;
  v.nodes = c->d_nodes;
  v.leaf_geo = c->d_leaf_geo;
  v.leaf_idx = c->d_leaf_idx;
  v.big_idx = c->d_big;
  v.n_nodes = c->n_nodes;
  v.n_big = c->n_big;
  v.n_leaf = c->n_leaf;
  v.walk0 = c->walk0;
  v.r_check = c->r_check;
  v.cell_start = c->d_cell_start;
  v.cell_items = c->d_cell_items;
  v.nb_word = c->d_nb_word;
  v.nb_items = c->d_nb_items;
  v.cell_rec = c->d_cell_rec;
  v.nb_rec = c->d_nb_rec;
  v.nb_c2 = 0.25 * c->pad * c->pad;
  if (c->tune.no_neighbors) v.nb_c2 = -1.0;  // C^2 <= -r^2 never holds
  // grid bounds / scale in FP32, as used: the cell index of the device is a
  // function of these exact float values, and the host places each sphere in
  // every cell its padded box overlaps under the SAME float cell boundaries
  for (int k = 0; k < 3; ++k) {
    v.glo[k] = c->pgrid.flo[k];
    v.ghi[k] = c->pgrid.fhi[k];
    v.gdims[k] = c->pgrid.dims[k];
  }
  v.ginv = c->pgrid.finv;
  v.gmargin = (float)(c->pad * 0.25);
  return v;
}

static int check_params(const rt_params* p) {
  if (!p) return set_error(RT_E_INVALID, "params is NULL");
  if (p->width < 2 || p->height < 2)
    return set_error(RT_E_INVALID, "width/height must be >= 2 (got %d x %d)", p->width, p->height);
  if (p->spp < 1) return set_error(RT_E_INVALID, "spp must be >= 1 (got %d)", p->spp);
  if (p->max_depth < -1 || p->max_depth > 100000)
    return set_error(RT_E_INVALID, "max_depth out of range (got %d)", p->max_depth);
  // row_offset >= height is a shard that owns no rows (more ranks than rows):
  // its render is empty
  if (p->row_stride < 1 || p->row_offset < 0)
    return set_error(RT_E_INVALID, "bad shard: row_offset %d row_stride %d height %d", p->row_offset,
                p->row_stride, p->height);
  if ((long long)p->width * p->height >= (1LL << 32))
    return set_error(RT_E_INVALID, "image too large for 32-bit pixel ids");
  if (p->flags & ~(RT_FLAG_NO_CULL | RT_FLAG_NO_FIXPOINT | RT_FLAG_NO_TAIL_PRIORITY |
                   RT_FLAG_CULL_STATS | RT_FLAG_MATERIALS))
    return set_error(RT_E_INVALID, "unknown flags 0x%x", p->flags);
  if ((p->flags & RT_FLAG_MATERIALS) && p->max_depth > psrt::kMatMaxDepth)
    return set_error(RT_E_INVALID, "max_depth %d above %d with RT_FLAG_MATERIALS", p->max_depth,
                     psrt::kMatMaxDepth);
  return RT_OK;
}

extern "C++" {  // psrt_error.h (rt_group_render's check)
int psrt::check_render_params(const void* p) { return check_params((const rt_params*)p); }
}

// Guided work queue (psrt_kernels.h TraceArgs::ph_*), BVH scenes. The first
// ticket size is the power of two <= total / (D x resident waves), clamped to
// [64, kWorkChunk]: a window takes ~77 loop iterations per 1024 units, so on a
// small launch (a strong-scaled shard) a large window of expensive pixels
// would outlast the rest of the launch. Working back from the end of the
// queue, each later phase halves the size (down to 64) and holds about K
// tickets per resident wave. Ticket ranges are contiguous: units a phase
// cannot fill with whole tickets carry into the next one. Tuning::queue_d /
// queue_k: tuning knobs.
// Small scenes (the linear sweep, ~5x cheaper rays) keep fixed tickets of
// kLinearChunk units: there the queue's atomics and the per-wave start-up
// cost more than the launch tail (C1: 0.31 ms with 1024-unit tickets on a few
// hundred waves vs 0.51 ms guided; C2 -7% guided).
static void queue_phases(psrt::TraceArgs& ta, int grid, bool guided, const psrt::Tuning& tu) {
  // two tickets per resident wave per phase (C3, 96 M units one frame at a
  // time: 13.64 -> 13.56 ms per step, r02), and the first ticket size at most
  // units / (2 x waves): the strong 1/8 shard's 20-frame launch (24 M units)
  // then starts with 1024-unit tickets instead of 512, and its trace takes
  // 1.480 instead of 1.503 ms per frame (r04, profiles/r04_queue; larger
  // launches are capped at 1024 either way)
  const double k = tu.queue_k;
  const double d = tu.queue_d;
  const uint64_t waves = (uint64_t)grid * (psrt::kTraceBlock / 64);
  unsigned s0 = guided ? psrt::kWorkChunk : psrt::kLinearChunk;
  if (tu.linear_chunk > 0 && !guided)
    s0 = std::max(64u, std::min(4096u, (unsigned)tu.linear_chunk));
  while (guided && s0 > 64 && (double)ta.total_units < d * (double)waves * (double)s0) s0 >>= 1;
  unsigned size[psrt::kQueuePhases];
  for (int p = 0; p < psrt::kQueuePhases; ++p) size[p] = guided ? std::max(64u, s0 >> p) : s0;
  uint64_t alloc[psrt::kQueuePhases], rem = ta.total_units;
  for (int p = psrt::kQueuePhases - 1; p >= 1; --p) {
    const uint64_t want = guided && size[p] < size[p - 1]
                              ? (uint64_t)(k * (double)waves * (double)size[p]) : 0;
    alloc[p] = std::min(rem, want);
    rem -= alloc[p];
  }
  alloc[0] = rem;
  uint64_t first = 0, base = 0, carry = 0;
  for (int p = 0; p < psrt::kQueuePhases; ++p) {
    ta.ph_first[p] = first;
    ta.ph_base[p] = base;
    ta.ph_size[p] = size[p];
    const uint64_t units = alloc[p] + carry;
    const uint64_t n = units / size[p];
    carry = units - n * size[p];
    first += n;
    base += n * size[p];
  }
  ta.ph_first[psrt::kQueuePhases] = ~0ull;
}

int rt_render_device(rt_context* c, const rt_params* p, double* d_accum, unsigned char* d_rgb8,
                     void* stream_) {
  return rt_render_device_frames(c, p, 1, d_accum ? &d_accum : nullptr,
                                 d_rgb8 ? &d_rgb8 : nullptr, stream_);
}

int rt_render_device_frames(rt_context* c, const rt_params* p, int nframes,
                            double* const* d_accum_f, unsigned char* const* d_rgb8_f,
                            void* stream_) {
  if (!c) return set_error(RT_E_INVALID, "rt_render_device: ctx is NULL");
  int rc = check_params(p);
  if (rc) return rc;
  if ((c->accum_pitch && c->accum_pitch < 3 * (size_t)p->width) ||
      (c->rgb8_pitch && c->rgb8_pitch < 3 * (size_t)p->width))
    return set_error(RT_E_INVALID, "row pitch (%zu doubles, %zu bytes) below 3 x width %d",
                     c->accum_pitch, c->rgb8_pitch, p->width);
  if ((c->accum_pitch || c->rgb8_pitch) && (p->flags & RT_FLAG_MATERIALS))
    return set_error(RT_E_INVALID, "row pitches are not supported with RT_FLAG_MATERIALS");
  if (nframes < 1 || nframes > psrt::kMaxFrames)
    return set_error(RT_E_INVALID, "rt_render_device_frames: nframes %d outside [1, %d]", nframes,
                     psrt::kMaxFrames);
  const size_t nf = (size_t)nframes;  // frames of the batch
  if (c->n < 0) return set_error(RT_E_SCENE, "rt_render_device: no scene set");
  // RT_FLAG_MATERIALS: the material integrator (psrt_mat.hip) over the
  // context's materials and lens camera; colour records of 3 doubles
  const bool mat = (p->flags & RT_FLAG_MATERIALS) != 0;
  if (mat && !c->has_mats)
    return set_error(RT_E_SCENE, "RT_FLAG_MATERIALS: no materials set for this scene");
  const size_t rec_bytes = mat ? psrt::kMatSampleBytes : psrt::kSampleBytes;
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t st = stream_ ? (hipStream_t)stream_ : c->stream;
  const int rows = rt_rows_owned(p->height, p->row_offset, p->row_stride);
  const size_t P = (size_t)rows * p->width;
  // The context's buffers (samples, counters, camera lists, events) are
  // shared by its renders: a render on another stream than the last one
  // starts after it (same stream: stream order already does it).
  if (c->in_flight && st != c->last_stream) HIP_TRY(hipStreamWaitEvent(st, c->ev_all1, 0));
  if (P == 0) {  // a shard that owns no rows: zero statistics, no launch
    const int qrc = quiesce(c);  // the last render's psrt_reduce writes h_stats
    if (qrc) return qrc;
    std::fill(c->h_stats, c->h_stats + psrt::kStatWords, 0ull);
    HIP_TRY(hipEventRecord(c->ev_all0, st));
    HIP_TRY(hipEventRecord(c->ev_all1, st));
    c->in_flight = true;
    c->last_stream = st;
    c->ev_used = 0;
    c->failed = false;
    c->last_mat = mat;
    c->last = rt_stats{};
    c->n_last = c->n;
    return RT_OK;
  }

  // sample chunking: the samples buffer holds s_chunk x P records of
  // kSampleBytes (t array, then k array), units < 2^32
  // (chunks of a multiple of 4 samples where possible: psrt_reduce then reads
  // 16-B aligned runs). The chunk count never changes a bit of the frame:
  // psrt_reduce continues each pixel's running sum across chunks, in sample
  // order (main.cc:77-84).
  const size_t s_units = ((1ULL << 32) - 1) / (P * nf);  // units of one launch < 2^32
  if (s_units < 1) return set_error(RT_E_INVALID, "shard too large");
  // The buffer is sized to the HBM actually free: hipMemGetInfo's free bytes
  // plus this context's current buffer (it is replaced), less a reserve for
  // the GPU's other users, capped by Tuning::sample_buf_mb.
  // The render's other buffers are decided first, so their growth comes out
  // of the same free HBM: the accumulator scratch (frames without a caller
  // accumulator, when the frame takes several chunks), the material path
  // scratch and the camera-ray lists.
  const bool use_bvh = c->bvh && !(p->flags & RT_FLAG_NO_CULL);
  // material kernel: the BVH staged in LDS when the workgroups resident per CU
  // stay as many as without (Tuning::mat_lds 0 / 1 forces it off / on)
  int mat_grid = use_bvh ? c->grid_mat_bvh : c->grid_mat;
  unsigned mat_lds = 0;
  if (mat && use_bvh) {
    const unsigned bytes = psrt::mat_lds_layout(c->n, c->n_nodes, c->n_leaf, c->n_big).bytes;
    int pc = 0;
    const double ml = c->tune.mat_lds;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&pc, psrt::psrt_trace_mat<true, true, false>,
                                                     psrt::kMatBlock, bytes) == hipSuccess &&
        pc >= 1 && (ml >= 0 ? ml != 0 : c->cus * pc >= c->grid_mat_bvh)) {
      mat_lds = bytes;
      mat_grid = c->cus * pc;
    }
  }
  const size_t mat_lanes = (size_t)mat_grid * psrt::kMatBlock;
  const size_t path_ints = mat ? mat_lanes * (size_t)std::max(1, p->max_depth) : 0;
  // camera-ray candidate lists: BVH scenes whose indices fit uint16 and whose
  // camera lies inside the range the pad covers (|o|_inf <= r_check)
  const double om = std::max(std::fabs(c->cam.origin[0]),
                             std::max(std::fabs(c->cam.origin[1]), std::fabs(c->cam.origin[2])));
  const bool camlist = !mat && use_bvh && c->n < (int)psrt::kCamOverflow && om <= c->r_check &&
                       !c->tune.no_camlist;
  // the material integrator's lists through the lens: the same conditions,
  // for the lens camera's origin
  const double lom = std::max(std::fabs(c->lcam.base.origin[0]),
                              std::max(std::fabs(c->lcam.base.origin[1]),
                                       std::fabs(c->lcam.base.origin[2])));
  const bool mat_list = mat && use_bvh && c->n < (int)psrt::kCamOverflow && lom <= c->r_check &&
                        !c->tune.no_camlist;
  bool any_null_acc = false;
  for (size_t f = 0; f < nf; ++f) any_null_acc = any_null_acc || !(d_accum_f && d_accum_f[f]);
  auto grow = [](size_t need, size_t have, size_t unit) { return need > have ? (need - have) * unit : 0; };
  const size_t other_bytes = (any_null_acc ? grow(nf * P * 3, c->accum_tmp_cap, sizeof(double)) : 0) +
                             grow(path_ints, c->path_cap, sizeof(int)) +
                             (camlist ? grow(P, c->plist_cap, sizeof(uint4)) : 0) +
                             (mat_list ? grow(P, c->mat_plist_cap, sizeof(uint4)) : 0);
  size_t cap_bytes = sample_buffer_cap_bytes(c->tune);
  // the current buffer already holds the whole render in one chunk: no query
  // (hipMemGetInfo is a host round trip on every render otherwise)
  const size_t recs_all = nf * P * (size_t)p->spp;
  const size_t need_all = mat ? 3 * recs_all : recs_all + (recs_all + 3) / 4;  // doubles
  const bool fits = c->d_samples && c->samples_cap >= need_all && (size_t)p->spp <= s_units &&
                    need_all * sizeof(double) <= cap_bytes && other_bytes == 0;
  if (!fits) {
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) == hipSuccess) {
      const size_t usable = fr + c->samples_cap * sizeof(double);
      const size_t keep = kHbmReserve + other_bytes;
      cap_bytes = std::min(cap_bytes, usable > keep ? usable - keep : 0);
    }
  }
  auto plan = [&](size_t s_max) {
    size_t sc = s_max;
    if (sc > 4) sc &= ~(size_t)3;
    if (sc < 1) sc = 1;
    if (sc > (size_t)p->spp) sc = p->spp;
    if (sc > s_units) sc = s_units > 4 ? s_units & ~(size_t)3 : s_units;
    // the same number of chunks, balanced (no short last chunk with its own tail)
    const size_t n = ((size_t)p->spp + sc - 1) / sc;
    if (n > 1) {
      size_t even = ((size_t)p->spp + n - 1) / n;
      if (even > 4) even = (even + 3) & ~(size_t)3;
      if (even <= sc) sc = even;
    }
    return sc;
  };
  size_t s_chunk = plan(cap_bytes / (nf * P * rec_bytes));
  // t array (doubles) then k array (uint16), P x s_chunk records each. If the
  // allocation still fails (another process took the memory meanwhile), halve
  // the chunk and try again.
  for (;;) {
    const size_t recs = nf * P * s_chunk;
    rc = ensure_buf(c, &c->d_samples, &c->samples_cap, mat ? 3 * recs : recs + (recs + 3) / 4);
    if (rc == RT_E_NOMEM && s_chunk > 1) {
      (void)hipGetLastError();  // clear the failed hipMalloc
      s_chunk = plan(s_chunk / 2);
      continue;
    }
    if (rc) return rc;
    break;
  }
  const int nchunks = (int)((p->spp + s_chunk - 1) / s_chunk);
  // per frame: its accumulators (a scratch block when the caller passes none
  // and the running sums must survive between sample chunks) and its bytes
  std::vector<double*> acc(nf, nullptr);
  std::vector<unsigned char*> rgb(nf, nullptr);
  bool need_tmp = false;
  for (size_t f = 0; f < nf; ++f) {
    acc[f] = d_accum_f ? d_accum_f[f] : nullptr;
    rgb[f] = d_rgb8_f ? d_rgb8_f[f] : nullptr;
    need_tmp = need_tmp || (!acc[f] && nchunks > 1);
  }
  if (need_tmp) {
    rc = ensure_buf(c, &c->d_accum_tmp, &c->accum_tmp_cap, nf * P * 3);
    if (rc) return rc;
    for (size_t f = 0; f < nf; ++f)
      if (!acc[f]) acc[f] = c->d_accum_tmp + f * P * 3;
  }
  rc = ensure_events(c, nchunks);
  if (rc) return rc;
  psrt::MatArgs ma{};
  if (mat) {  // the path scratch: one column per resident lane, max_depth rows
    const size_t lanes = mat_lanes;
    const size_t need_ints = path_ints;
    if (c->path_cap < need_ints) {
      rc = quiesce(c);
      if (rc) return rc;
      (void)hipFree(c->d_path);
      c->d_path = nullptr;
      c->path_cap = 0;
      HIP_TRY(hipMalloc(&c->d_path, need_ints * sizeof(int)));
      c->path_cap = need_ints;
    }
    ma.n = c->n;
    for (int k = 0; k < 3; ++k) {
      ma.org[k] = c->lcam.base.origin[k];
      ma.llc[k] = c->lcam.base.lower_left[k];
      ma.hor[k] = c->lcam.base.horizontal[k];
      ma.ver[k] = c->lcam.base.vertical[k];
      ma.lu[k] = c->lcam.u[k];
      ma.lv[k] = c->lcam.v[k];
    }
    ma.lens_radius = c->lcam.lens_radius;
    ma.width = p->width;
    ma.height = p->height;
    ma.max_depth = p->max_depth;
    ma.row_offset = p->row_offset;
    ma.row_stride = p->row_stride;
    ma.pixels = (unsigned)P;
    ma.frames = nframes;
    for (int f = 0; f < nframes; ++f) ma.seedmix[f] = splitmix64_host(p->seed + (uint64_t)f);
    ma.div_p = fast_div_make((unsigned)P);
    ma.div_w = fast_div_make((unsigned)p->width);
    ma.work_counter = c->d_counters + kHeads;
    ma.ray_counter = c->d_counters + kSets;
    ma.mats = c->d_mats;
    ma.path = c->d_path;
    ma.path_stride = (unsigned)lanes;
    ma.batch = (unsigned)std::max(1.0, c->tune.mat_batch);
  }

  psrt::TraceArgs ta{};
  ta.n = c->n;
  for (int k = 0; k < 3; ++k) {
    ta.org[k] = c->cam.origin[k];
    ta.llc[k] = c->cam.lower_left[k];
    ta.hor[k] = c->cam.horizontal[k];
    ta.ver[k] = c->cam.vertical[k];
  }
  ta.width = p->width;
  ta.height = p->height;
  ta.max_depth = p->max_depth;
  ta.row_offset = p->row_offset;
  ta.row_stride = p->row_stride;
  ta.pixels = (unsigned)P;
  ta.frames = nframes;
  for (int f = 0; f < nframes; ++f) ta.seedmix[f] = splitmix64_host(p->seed + (uint64_t)f);
  ta.div_p = fast_div_make((unsigned)P);
  ta.tail_prio = !(p->flags & RT_FLAG_NO_TAIL_PRIORITY);
  ta.div_w = fast_div_make((unsigned)p->width);
  ta.work_counter = c->d_counters + kHeads;
  ta.ray_counter = c->d_counters + kSets;
  ta.drain_flag = c->d_drain;

  // No memset here: the queue heads and counter sets are zero (context
  // creation, then every psrt_reduce), and a small fill kernel on this stream
  // would wait for a CU slot behind another frame's persistent launch.
  const bool stamps = !mat && c->tune.stamps != 0;  // the diagnostic variant
  if (stamps) HIP_TRY(hipMemsetAsync(c->d_counters + 8, 0, 120 * sizeof(unsigned long long), st));
  ta.stamps = c->d_counters + 8;
  ta.wave_log = nullptr;
  if (stamps) {
    const size_t need = (size_t)std::max(c->grid, c->grid_bvh) * (psrt::kTraceBlock / 64) * 5;
    if (c->wave_log_cap < need) {
      rc = quiesce(c);
      if (rc) return rc;
      (void)hipFree(c->d_wave_log);
      c->d_wave_log = nullptr;
      c->wave_log_cap = 0;
      HIP_TRY(hipMalloc(&c->d_wave_log, need * sizeof(unsigned long long)));
      c->wave_log_cap = need;
    }
    HIP_TRY(hipMemsetAsync(c->d_wave_log, 0, need * sizeof(unsigned long long), st));
    ta.wave_log = c->d_wave_log;
    c->wave_log_used = need / 5;
  }
  {
    // (the loop schedule: kRefillMin, kWalkBatch, kWalkTail, kRngFill,
    // kRngExtra in psrt_kernels.hip, compile-time since r03)
    // The kernel's per-lane counters are 32-bit; a lane flushes them in its
    // wave's refill block once one reaches flush_at, and between two such
    // blocks it adds at most one sample's work: <= max_depth + 1 rays (so
    // `rays` is always exact), <= (max_depth + 1)(4n + 16) sphere / box tests
    // (hint + big + list <= 2n + 16, leaves <= n; box tests <= 2 per node).
    // flush_at leaves that much headroom below 2^32 (the test counts stay exact
    // while one sample's tests are < 2^32). Tuning::flush_at: test knob, >= 1.
    const uint64_t per_sample = (uint64_t)(p->max_depth + 1) * (4ull * (uint64_t)c->n + 16ull);
    const uint64_t room = per_sample < 0xFFFFFFFFull ? 0xFFFFFFFFull - per_sample : 1ull;
    ta.flush_at = (unsigned)std::max<uint64_t>(1ull, std::min<uint64_t>(room, 0x80000000ull));
    if (c->tune.flush_at >= 1 && c->tune.flush_at < ta.flush_at)
      ta.flush_at = (unsigned)c->tune.flush_at;
  }
  psrt::BvhView bv = bvh_view(c);
  bv.fixpoint = !(p->flags & RT_FLAG_NO_FIXPOINT) && !c->tune.no_fixpoint;
  if (mat_list && c->mat_plist_cap < P) {
    rc = quiesce(c);
    if (rc) return rc;
    (void)hipFree(c->d_mat_plist);
    c->d_mat_plist = nullptr;
    c->mat_plist_cap = 0;
    HIP_TRY(hipMalloc(&c->d_mat_plist, P * sizeof(uint4)));
    c->mat_plist_cap = P;
    c->mat_plist_valid = false;
  }
  if (camlist && c->plist_cap < P) {
    rc = quiesce(c);
    if (rc) return rc;
    (void)hipFree(c->d_plist);
    c->d_plist = nullptr;
    c->plist_cap = 0;
    HIP_TRY(hipMalloc(&c->d_plist, P * sizeof(uint4)));
    c->plist_cap = P;
    c->plist_valid = false;
  }
  if (c->dirty) {  // an earlier render failed part-way: heads and sets back to zero
    HIP_TRY(hipMemsetAsync(c->d_counters + kHeads, 0,
                           (kCounterWords - kHeads) * sizeof(unsigned long long), st));
    c->dirty = false;
  }
  HIP_TRY(hipEventRecord(c->ev_all0, st));
  const int key[4] = {p->width, p->height, p->row_offset, p->row_stride};
  if (camlist && c->plist_valid && std::equal(key, key + 4, c->plist_key)) {
    HIP_TRY(hipStreamWaitEvent(st, c->ev_plist, 0));  // built on another stream, maybe
    bv.plist = c->d_plist;
  } else if (camlist) {
    psrt::CamListArgs la{};
    for (int k = 0; k < 3; ++k) {
      la.org[k] = c->cam.origin[k];
      la.llc[k] = c->cam.lower_left[k];
      la.hor[k] = c->cam.horizontal[k];
      la.ver[k] = c->cam.vertical[k];
    }
    la.width = p->width;
    la.height = p->height;
    la.row_offset = p->row_offset;
    la.row_stride = p->row_stride;
    la.rows = rows;
    la.leaf_geo = c->d_leaf_geo;
    la.leaf_idx = c->d_leaf_idx;
    la.n_leaf = c->n_leaf;
    la.pad = c->pad;
    la.plist = c->d_plist;
    const dim3 lg((p->width + psrt::kCamTile - 1) / psrt::kCamTile,
                  (rows + psrt::kCamTile - 1) / psrt::kCamTile);
    hipLaunchKernelGGL(psrt::psrt_camera_lists, lg, dim3(64), 0, st, la);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(c->ev_plist, st));
    std::copy(key, key + 4, c->plist_key);
    c->plist_valid = true;
    bv.plist = c->d_plist;
  }
  if (mat_list && c->mat_plist_valid && std::equal(key, key + 4, c->mat_plist_key)) {
    HIP_TRY(hipStreamWaitEvent(st, c->ev_mat_plist, 0));
    ma.plist = c->d_mat_plist;
  } else if (mat_list) {
    psrt::MatCamListArgs la{};
    for (int k = 0; k < 3; ++k) {
      la.org[k] = c->lcam.base.origin[k];
      la.llc[k] = c->lcam.base.lower_left[k];
      la.hor[k] = c->lcam.base.horizontal[k];
      la.ver[k] = c->lcam.base.vertical[k];
    }
    la.lens_radius = std::fabs(c->lcam.lens_radius);
    la.width = p->width;
    la.height = p->height;
    la.row_offset = p->row_offset;
    la.row_stride = p->row_stride;
    la.rows = rows;
    la.leaf_geo = c->d_leaf_geo;
    la.leaf_idx = c->d_leaf_idx;
    la.n_leaf = c->n_leaf;
    la.pad = c->pad;
    la.plist = c->d_mat_plist;
    const dim3 lg((p->width + psrt::kCamTile - 1) / psrt::kCamTile,
                  (rows + psrt::kCamTile - 1) / psrt::kCamTile);
    hipLaunchKernelGGL(psrt::psrt_mat_camera_lists, lg, dim3(64), 0, st, la);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(c->ev_mat_plist, st));
    std::copy(key, key + 4, c->mat_plist_key);
    c->mat_plist_valid = true;
    ma.plist = c->d_mat_plist;
  }
  // A HIP failure after the first trace launch would leave the queue heads and
  // counter sets non-zero (only psrt_reduce re-zeroes them): the context is
  // marked dirty, the enqueued part is fenced by ev_all1 like a whole render,
  // and the next render re-zeroes them with a stream-ordered memset first.
  c->dirty = true;
  // fault injection (rt_debug_fail_after_trace, tests only): fail after chunk
  // k's trace launch and before its reduce, as a HIP error there would; one shot
  const int fail_at = c->fail_after;
  c->fail_after = -1;
  auto enqueue_chunks = [&]() -> int {
  for (int ch = 0; ch < nchunks; ++ch) {
    const int s0 = (int)(ch * s_chunk);
    const int sc = (int)std::min<size_t>(s_chunk, (size_t)(p->spp - s0));
    ta.s_begin = s0;
    ta.s_count = sc;
    ta.div_s = fast_div_make((unsigned)sc);
    ta.total_units = (uint64_t)nf * P * sc;
    const size_t fu = P * (size_t)sc;  // units (records) of one frame in this chunk
    if (mat) {
      ma.s_begin = s0;
      ma.s_count = sc;
      ma.div_s = ta.div_s;
      ma.total_units = ta.total_units;
      HIP_TRY(hipEventRecord(c->ev[2 * ch], st));
      // RT_FLAG_CULL_STATS: the variant that counts the sphere / box tests
      auto mlaunch = [&](auto kern, unsigned lds_bytes) {
        hipLaunchKernelGGL(kern, dim3(mat_grid), dim3(psrt::kMatBlock), lds_bytes, st, c->d_geo,
                           c->d_inv_r, c->d_samples, ma, bv);
      };
      const bool mcount = (p->flags & RT_FLAG_CULL_STATS) != 0;
      if (mat_lds)
        mcount ? mlaunch(psrt::psrt_trace_mat<true, true, true>, mat_lds)
               : mlaunch(psrt::psrt_trace_mat<true, true, false>, mat_lds);
      else if (use_bvh)
        mcount ? mlaunch(psrt::psrt_trace_mat<true, false, true>, 0)
               : mlaunch(psrt::psrt_trace_mat<true, false, false>, 0);
      else
        mcount ? mlaunch(psrt::psrt_trace_mat<false, false, true>, 0)
               : mlaunch(psrt::psrt_trace_mat<false, false, false>, 0);
      HIP_TRY(hipGetLastError());
      HIP_TRY(hipEventRecord(c->ev[2 * ch + 1], st));
      if (ch == fail_at)
        return set_error(RT_E_HIP, "rt_debug_fail_after_trace: failure injected after chunk %d", ch);
      for (size_t f = 0; f < nf; ++f) {
        psrt::ReduceArgs ra{};
        ra.samp_t = c->d_samples + 3 * f * fu;
        ra.pixels = (unsigned)P;
        ra.s_count = sc;
        ra.first_chunk = ch == 0;
        ra.spp_total = p->spp;
        ra.accum = acc[f];
        ra.rgb8 = (ch == nchunks - 1) ? rgb[f] : nullptr;
        ra.fold_stats = f == 0;
        ra.heads = c->d_counters + kHeads;
        ra.sets = c->d_counters + kSets;
        ra.totals = c->d_counters + kTotals;
        ra.host_stats = (ch == nchunks - 1 && f == 0) ? c->d_stats : nullptr;
        const unsigned blocks = (unsigned)((P + psrt::kReduceBlock - 1) / psrt::kReduceBlock);
        hipLaunchKernelGGL(psrt::psrt_reduce_rgb, dim3(blocks), dim3(psrt::kReduceBlock), 0, st,
                           ra);
        HIP_TRY(hipGetLastError());
      }
      continue;
    }
    queue_phases(ta, use_bvh ? c->grid_bvh : c->grid, use_bvh, c->tune);
    HIP_TRY(hipEventRecord(c->ev[2 * ch], st));
    const double4* g4 = c->d_geo;
    const double* ir = c->d_inv_r;
    const dim3 blk(psrt::kTraceBlock);
    // scene data in LDS when three workgroups per CU still fit (the BVH
    // kernel's resident count otherwise: its global-memory variant)
    const unsigned lds_bytes = psrt::lds_layout(c->n, c->n_nodes, c->n_leaf, c->n_big).bytes;
    const bool lds = use_bvh && lds_bytes <= c->lds_max && !c->tune.no_lds;
    // Tuning::blocks_per_cu: measurement knob (occupancy sweep), 0 = resident max
    const int bpc = (int)c->tune.blocks_per_cu;
    auto launch = [&](auto kern, int grid) {
      if (bpc > 0) grid = std::min(grid, std::max(1, c->cus * bpc));
      hipLaunchKernelGGL(kern, dim3(grid), blk, lds ? lds_bytes : 0, st, g4, ir, c->d_samples, ta,
                         bv);
    };
    // RT_FLAG_CULL_STATS: the variant that counts sphere / box tests
    auto pick = [&](auto kBVH, auto kStamps, auto kLds, int grid) {
      if (p->flags & RT_FLAG_CULL_STATS)
        launch(psrt::psrt_trace<decltype(kBVH)::value, decltype(kStamps)::value,
                                decltype(kLds)::value, true>, grid);
      else
        launch(psrt::psrt_trace<decltype(kBVH)::value, decltype(kStamps)::value,
                                decltype(kLds)::value, false>, grid);
    };
    using T = std::true_type;
    using F = std::false_type;
    ta.drain_epoch = c->drain_epoch + 1;  // counted once the launch is enqueued
    if (!use_bvh)
      stamps ? pick(F{}, T{}, F{}, c->grid) : pick(F{}, F{}, F{}, c->grid);
    else if (lds)
      stamps ? pick(T{}, T{}, T{}, c->grid_bvh) : pick(T{}, F{}, T{}, c->grid_bvh);
    else
      stamps ? pick(T{}, T{}, F{}, c->grid_bvh) : pick(T{}, F{}, F{}, c->grid_bvh);
    HIP_TRY(hipGetLastError());
    c->drain_epoch = ta.drain_epoch;
    HIP_TRY(hipEventRecord(c->ev[2 * ch + 1], st));
    if (ch == fail_at)
      return set_error(RT_E_HIP, "rt_debug_fail_after_trace: failure injected after chunk %d", ch);
    // psrt_reduce: frames whose accumulators and bytes are evenly strided
    // (the bench's, torch's [B, rows, W, 3] blocks) are reduced by ONE launch
    // (blockIdx.y = frame: the frames' reduces overlap instead of running back
    // to back with a launch gap each); other pointer sets by one launch per
    // frame. Frame 0's block 0 also folds the launch's counter sets into the
    // render's totals and re-zeroes the queue heads.
    const bool last = ch == nchunks - 1;
    auto strided = [&](auto* const* v, size_t& stride) {
      stride = 0;
      if (nf == 1) return true;
      for (size_t f = 0; f < nf; ++f)
        if ((v[f] == nullptr) != (v[0] == nullptr)) return false;
      if (!v[0]) return true;
      const ptrdiff_t d = v[1] - v[0];
      if (d <= 0) return false;
      for (size_t f = 1; f < nf; ++f)
        if (v[f] - v[f - 1] != d) return false;
      stride = (size_t)d;
      return true;
    };
    size_t acc_stride = 0, rgb_stride = 0;
    std::vector<unsigned char*> rgb_now(nf, nullptr);
    for (size_t f = 0; f < nf; ++f) rgb_now[f] = last ? rgb[f] : nullptr;
    // one launch reduces the frames concurrently: only when no two frames'
    // buffers overlap (a stride of at least one frame); overlapping buffers
    // keep the per-frame launches, in frame order
    // a frame's footprint: its rows, row pitches apart (rt_context_set_row_pitch)
    const size_t W3 = 3 * (size_t)p->width;
    const size_t apitch = c->accum_pitch ? c->accum_pitch : W3;
    const size_t rpitch = c->rgb8_pitch ? c->rgb8_pitch : W3;
    const size_t acc_span = rows > 0 ? (size_t)(rows - 1) * apitch + W3 : 0;
    const size_t rgb_span = rows > 0 ? (size_t)(rows - 1) * rpitch + W3 : 0;
    const bool one = strided(acc.data(), acc_stride) && strided(rgb_now.data(), rgb_stride) &&
                     (nf == 1 || ((acc_stride == 0 || acc_stride >= acc_span) &&
                                  (rgb_stride == 0 || rgb_stride >= rgb_span)));
    for (size_t f0 = 0; f0 < nf; f0 += one ? nf : 1) {
      psrt::ReduceArgs ra{};
      ra.samp_t = c->d_samples + f0 * fu;
      // the k array follows the t array of all frames
      ra.samp_k = (const unsigned short*)(c->d_samples + nf * fu) + f0 * fu;
      ra.pixels = (unsigned)P;
      ra.s_count = sc;
      ra.first_chunk = ch == 0;
      ra.spp_total = p->spp;
      ra.accum = acc[f0];
      ra.rgb8 = rgb_now[f0];
      ra.frame_units = fu;
      ra.accum_stride = acc_stride;
      ra.rgb8_stride = rgb_stride;
      ra.accum_pitch = apitch == W3 ? 0 : apitch;
      ra.rgb8_pitch = rpitch == W3 ? 0 : rpitch;
      ra.width = (unsigned)p->width;
      ra.fold_stats = f0 == 0;
      ra.fast_k = p->max_depth <= 1000;
      ra.heads = c->d_counters + kHeads;
      ra.sets = c->d_counters + kSets;
      ra.totals = c->d_counters + kTotals;
      ra.host_stats = (last && f0 == 0) ? c->d_stats : nullptr;
      const unsigned blocks = (unsigned)((P + psrt::kReduceBlock - 1) / psrt::kReduceBlock);
      // Tuning::reduce_lean (frames in flight): the variant that fits beside a
      // resident trace launch, when its register count allows (lean_ok)
      const bool lean = c->tune.reduce_lean != 0 && ra.fast_k && sc % 4 == 0 && c->lean_ok;
      ra.inv_spp = 1.0 / (double)p->spp;
      if (lean && ra.fold_stats)  // the fold psrt_reduce_lean leaves out
        hipLaunchKernelGGL(psrt::psrt_fold_stats, dim3(1), dim3(64), 0, st, ra);
      hipLaunchKernelGGL(lean ? psrt::psrt_reduce_lean : psrt::psrt_reduce,
                         dim3(blocks, one ? (unsigned)nf : 1u), dim3(psrt::kReduceBlock), 0, st, ra);
      HIP_TRY(hipGetLastError());
    }
  }
  return RT_OK;
  };
  rc = enqueue_chunks();
  const hipError_t fence = hipEventRecord(c->ev_all1, st);
  c->in_flight = fence == hipSuccess;
  c->last_stream = st;
  c->last_mat = mat;
  c->last_stamps = stamps;
  if (rc) {
    // a failed render's timings are not reported: no event pair is summed
    // (kernel_ms and total_ms read 0 until the next successful render)
    c->ev_used = 0;
    c->failed = true;
    c->last = rt_stats{};
    return rc;
  }
  if (fence != hipSuccess)
    return set_error(RT_E_HIP, "hipEventRecord: %s", hipGetErrorString(fence));
  c->dirty = false;
  c->failed = false;
  c->ev_used = nchunks;
  c->last = rt_stats{};
  c->last.samples = (uint64_t)nf * P * p->spp;
  c->n_last = c->n;
  return RT_OK;
}

void* rt_context_stream(rt_context* c) { return c ? (void*)c->stream : nullptr; }

int rt_context_sync_stats(rt_context* c, rt_stats* s) {
  if (!c) return set_error(RT_E_INVALID, "rt_context_sync_stats: ctx is NULL");
  if (!c->in_flight) {  // nothing rendered yet: zero counters (ABI 2 behaviour)
    if (s) *s = rt_stats{};
    return RT_OK;
  }
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipEventSynchronize(c->ev_all1));
  if (c->failed) {  // waited for the enqueued part; a failed render reports nothing
    c->last = rt_stats{};
    if (s) *s = c->last;
    return RT_OK;
  }
  // the render's last psrt_reduce wrote its totals into pinned host memory
  unsigned long long cnt[psrt::kStatWords];
  for (int k = 0; k < psrt::kStatWords; ++k) cnt[k] = ((volatile unsigned long long*)c->h_stats)[k];
  const unsigned long long rays = cnt[0];
  double kms = 0.0;
  for (int ch = 0; ch < c->ev_used; ++ch) {
    float ms = 0.f;
    HIP_TRY(hipEventElapsedTime(&ms, c->ev[2 * ch], c->ev[2 * ch + 1]));
    kms += ms;
  }
  float all = 0.f;
  HIP_TRY(hipEventElapsedTime(&all, c->ev_all0, c->ev_all1));
  c->last.rays = rays;
  c->last.sphere_tests = rays * (uint64_t)(c->n_last > 0 ? c->n_last : 0);
  c->last.tests_executed = cnt[1];
  c->last.box_tests = cnt[2];
  c->last.rays_traced = cnt[3];
  c->last.prerejects = cnt[4];
  c->last.root_box_tests = cnt[5];
  c->last.kernel_ms = kms;
  c->last.total_ms = all;
  if (c->last_stamps) {  // the diagnostic variant's section clocks and probes
    unsigned long long sec[60];
    HIP_TRY(hipMemcpy(sec, c->d_counters + 8, sizeof sec, hipMemcpyDeviceToHost));
    static const char* names[24] = {"refill", "store", "hit", "hint", "nb", "cam",
                                    "grid", "walk", "trial", "scatter", "hint_hit",
                                    "hint_tiny", "grid_cell", "grid_out", "grid_none_fin",
                                    "grid_none_inf", "far_miss", "park", "list_trip",
                                    "walk_bvh", "walk_big", "walk_miss", "walk_fin", "walk_inf"};
    std::string u = "{\"psrt_util\": {";
    for (int k = 0; k < 24; ++k) {
      char b[128];
      const double w = (double)sec[12 + 2 * k], l = (double)sec[13 + 2 * k];
      std::snprintf(b, sizeof b, "%s\"%s\": [%.4g, %.2f]", k ? ", " : "", names[k], w,
                    w > 0 ? l / w : 0.0);
      u += b;
    }
    std::fprintf(stderr, "%s}}\n", u.c_str());
    if (c->d_wave_log && c->wave_log_used) {
      // wave timeline of the last launch: start, queue-empty and exit times
      // relative to the first start, percentiles over waves, in microseconds
      std::vector<unsigned long long> wl(c->wave_log_used * 5);
      HIP_TRY(hipMemcpy(wl.data(), c->d_wave_log, wl.size() * sizeof(unsigned long long),
                        hipMemcpyDeviceToHost));
      unsigned long long t0 = ~0ull;
      for (size_t w = 0; w < c->wave_log_used; ++w)
        if (wl[5 * w]) t0 = std::min(t0, wl[5 * w]);
      std::vector<double> st_, ex, en, it_ex, it_dr;
      for (size_t w = 0; w < c->wave_log_used; ++w) {
        const unsigned long long* e = &wl[5 * w];
        if (!e[0]) continue;
        st_.push_back((e[0] - t0) * 0.01);
        if (e[1]) {
          ex.push_back((e[1] - t0) * 0.01);
          it_ex.push_back((double)e[3]);
          it_dr.push_back((double)(e[4] - e[3]));
        }
        en.push_back((e[2] - t0) * 0.01);
      }
      auto pct = [](std::vector<double> v) {
        std::string r = "[";
        if (!v.empty()) {
          std::sort(v.begin(), v.end());
          const double q[6] = {0, 0.1, 0.5, 0.9, 0.99, 1.0};
          for (int k = 0; k < 6; ++k) {
            char b[32];
            std::snprintf(b, sizeof b, "%s%.1f", k ? ", " : "", v[(size_t)(q[k] * (v.size() - 1))]);
            r += b;
          }
        }
        return r + "]";
      };
      std::fprintf(stderr,
                   "{\"psrt_waves\": {\"waves\": %zu, \"pct\": [0, 10, 50, 90, 99, 100], "
                   "\"start_us\": %s, \"queue_empty_us\": %s, \"exit_us\": %s, "
                   "\"iters_to_empty\": %s, \"drain_iters\": %s}}\n",
                   st_.size(), pct(st_).c_str(), pct(ex).c_str(), pct(en).c_str(),
                   pct(it_ex).c_str(), pct(it_dr).c_str());
    }
    double tot = 0;
    for (int k = 0; k < 8; ++k) tot += (double)sec[k];
    std::fprintf(stderr,
                 "{\"psrt_sections\": {\"refill\": %.4f, \"hit_quick\": %.4f, "
                 "\"q_hint\": %.4f, \"q_big\": %.4f, \"q_grid\": %.4f, \"scatter\": %.4f, "
                 "\"fill_shade\": %.4f, \"traverse\": %.4f, \"wave_cycles\": %.4g, "
                 "\"wave_trips\": %llu, \"wave_leaf_trips\": %llu, \"trav_rays\": %llu, "
                 "\"lane_boxes\": %llu, \"leaf_visits\": %llu, \"rays\": %llu}}\n",
                 sec[0] / tot, sec[1] / tot, sec[5] / tot, sec[6] / tot, sec[7] / tot,
                 sec[2] / tot, sec[3] / tot, sec[4] / tot, tot, sec[8], sec[9], sec[10],
                 (unsigned long long)cnt[2], sec[11], (unsigned long long)rays);
  }
  if (s) *s = c->last;
  return RT_OK;
}

int rt_quantize_device(rt_context* c, const double* d_accum, int width, int rows, int spp,
                       unsigned char* d_rgb8, void* stream_) {
  if (!c || !d_accum || !d_rgb8 || width <= 0 || rows < 0 || spp <= 0)
    return set_error(RT_E_INVALID, "rt_quantize_device: bad arguments");
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t st = stream_ ? (hipStream_t)stream_ : c->stream;
  const size_t n = (size_t)width * rows * 3;
  if (n == 0) return RT_OK;
  hipLaunchKernelGGL(psrt::psrt_quantize, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                     d_accum, d_rgb8, (unsigned)n, spp);
  HIP_TRY(hipGetLastError());
  return RT_OK;
}

// The device address of page-locked host memory at p (rt_host_alloc,
// hipHostMalloc, hipHostRegister), or nullptr for pageable memory: the
// render's last kernels then write the caller's frame directly.
static void* mapped_host(const void* p) {
  if (!p) return nullptr;
  hipPointerAttribute_t at{};
  if (hipPointerGetAttributes(&at, p) != hipSuccess) {
    (void)hipGetLastError();  // pageable memory: not an error of the render
    return nullptr;
  }
  return at.type == hipMemoryTypeHost ? at.devicePointer : nullptr;
}

// One render of a one-shot entry into the caller's host buffers. Page-locked
// buffers (rt_host_alloc) are the render's own outputs: psrt_reduce writes
// the sums and bytes across the link as it forms them. Pageable ones receive
// the device frame by copy (HIP stages it through its own pinned buffers).
static int render_to_host(rt_context* c, const rt_params* p, double* accum_rgb,
                          unsigned char* rgb8, rt_stats* stats) {
  const int rows = rt_rows_owned(p->height, p->row_offset, p->row_stride);
  const size_t P = rows > 0 ? (size_t)rows * p->width : 0;
  double* h_acc = (double*)mapped_host(accum_rgb);
  unsigned char* h_rgb = (unsigned char*)mapped_host(rgb8);
  double* d_acc = h_acc;
  unsigned char* d_rgb = h_rgb;
  if ((accum_rgb && !h_acc) || (rgb8 && !h_rgb) || !accum_rgb) {
    // the device frame (the running sums live on the device whenever the
    // caller's are not device-visible or not wanted)
    int rc = ensure_buf(c, &c->d_accum_tmp, &c->accum_tmp_cap, P * 3 + (P * 3 + 7) / 8 + 1);
    if (rc) return rc;
    if (!h_acc) d_acc = c->d_accum_tmp;
    if (!h_rgb) d_rgb = (unsigned char*)(c->d_accum_tmp + P * 3);
  }
  int rc = rt_render_device(c, p, d_acc, rgb8 ? d_rgb : nullptr, nullptr);
  if (rc) return rc;
  if (accum_rgb && P && !h_acc)
    HIP_TRY(hipMemcpyAsync(accum_rgb, d_acc, P * 3 * sizeof(double), hipMemcpyDeviceToHost,
                           c->stream));
  if (rgb8 && P && !h_rgb)
    HIP_TRY(hipMemcpyAsync(rgb8, d_rgb, P * 3, hipMemcpyDeviceToHost, c->stream));
  rc = rt_context_sync_stats(c, stats);  // waits for the render (and its copies)
  if (rc) return rc;
  HIP_TRY(hipStreamSynchronize(c->stream));
  return RT_OK;
}

// The default context of RT_DEVICE, returned with that device's lock held
// in *lock: the one-shot entries run whole under it, so host threads calling
// them on one device take turns instead of sharing buffers mid-call.
static int get_default_context(rt_context** out, std::unique_lock<std::mutex>* lock) {
  const int dev = default_device();
  if (dev < 0 || dev >= 64) return set_error(RT_E_INVALID, "RT_DEVICE out of range");
  *lock = std::unique_lock<std::mutex>(g_device_mu[dev]);
  std::lock_guard<std::mutex> lk(g_default_mu);
  if (!g_default[dev]) {
    int rc = rt_context_create(dev, &g_default[dev]);
    if (rc) return rc;
  }
  *out = g_default[dev];
  (*out)->tune = tuning_defaults();  // the process defaults at each one-shot call
  return RT_OK;
}

int rt_context_wait_drain(const rt_context* c, void* stream) {
  if (!c) return set_error(RT_E_INVALID, "rt_context_wait_drain: ctx is NULL");
  if (!c->d_drain)
    return set_error(RT_E_HIP, "rt_context_wait_drain: no drain flag (signal memory unavailable)");
  if (c->drain_epoch == 0) return RT_OK;  // nothing enqueued to wait for
  HIP_TRY(hipSetDevice(c->device));
  // the epoch of the context's last enqueued trace launch: set by its waves
  // (a launch always empties its queue), and never lowered afterwards
  HIP_TRY(hipStreamWaitValue64((hipStream_t)stream, c->d_drain, c->drain_epoch,
                               hipStreamWaitValueGte));
  return RT_OK;
}

int rt_context_set_row_pitch(rt_context* c, size_t accum_pitch, size_t rgb8_pitch) {
  if (!c) return set_error(RT_E_INVALID, "rt_context_set_row_pitch: ctx is NULL");
  HIP_TRY(hipSetDevice(c->device));
  {  // renders already enqueued keep the layout they were enqueued with
    const int rc = quiesce(c);
    if (rc) return rc;
  }
  c->accum_pitch = accum_pitch;
  c->rgb8_pitch = rgb8_pitch;
  return RT_OK;
}

int rt_host_register(void* p, size_t bytes) {
  if (!p || !bytes) return set_error(RT_E_INVALID, "rt_host_register: bad arguments");
  const hipError_t e =
      hipHostRegister(p, bytes, hipHostRegisterPortable | hipHostRegisterMapped);
  if (e != hipSuccess)
    return set_error(e == hipErrorOutOfMemory ? RT_E_NOMEM : RT_E_HIP, "rt_host_register(%zu): %s",
                     bytes, hipGetErrorString(e));
  return RT_OK;
}

int rt_host_unregister(void* p) {
  if (!p) return RT_OK;
  HIP_TRY(hipHostUnregister(p));
  return RT_OK;
}

int rt_host_alloc(size_t bytes, void** out) {
  if (!out) return set_error(RT_E_INVALID, "rt_host_alloc: out is NULL");
  *out = nullptr;
  if (bytes == 0) return RT_OK;
  const hipError_t e = hipHostMalloc(out, bytes, hipHostMallocPortable | hipHostMallocMapped);
  if (e != hipSuccess) {
    *out = nullptr;
    return set_error(e == hipErrorOutOfMemory ? RT_E_NOMEM : RT_E_HIP,
                     "rt_host_alloc(%zu): %s", bytes, hipGetErrorString(e));
  }
  return RT_OK;
}

int rt_host_free(void* p) {
  if (!p) return RT_OK;
  HIP_TRY(hipHostFree(p));
  return RT_OK;
}

int rt_render(const rt_sphere* sph, int n, const rt_camera* cam, const rt_params* p,
              double* accum_rgb, unsigned char* rgb8, rt_stats* stats) {
  if (!cam || !p || n < 0 || (n > 0 && !sph))
    return set_error(RT_E_INVALID, "rt_render: bad arguments");
  int rc = check_params(p);
  if (rc) return rc;
  // an empty shard (row_offset >= height) may pass no output buffers
  if (!accum_rgb && !rgb8 && rt_rows_owned(p->height, p->row_offset, p->row_stride) > 0)
    return set_error(RT_E_INVALID, "rt_render: no output buffer");
  rt_context* c = nullptr;
  std::unique_lock<std::mutex> lk;
  rc = get_default_context(&c, &lk);
  if (rc) return rc;
  rc = rt_context_set_scene(c, sph, n, cam);
  if (rc) return rc;
  return render_to_host(c, p, accum_rgb, rgb8, stats);
}

int rt_context_set_materials(rt_context* c, const rt_material* mats, int n,
                             const rt_camera_lens* cam) {
  if (!c) return set_error(RT_E_INVALID, "rt_context_set_materials: ctx is NULL");
  if (!mats) {
    c->has_mats = false;
    return RT_OK;
  }
  if (!cam) return set_error(RT_E_INVALID, "rt_context_set_materials: cam is NULL");
  if (c->n < 0) return set_error(RT_E_SCENE, "rt_context_set_materials: no scene set");
  if (n != c->n)
    return set_error(RT_E_INVALID, "rt_context_set_materials: %d materials for %d spheres", n, c->n);
  std::vector<psrt::DevMaterial> dm((size_t)std::max(1, n));
  for (int k = 0; k < n; ++k) {
    const rt_material& m = mats[k];
    if (m.kind != RT_MAT_LAMBERTIAN && m.kind != RT_MAT_METAL && m.kind != RT_MAT_DIELECTRIC)
      return set_error(RT_E_INVALID, "rt_context_set_materials: material %d has kind %d", k, m.kind);
    psrt::DevMaterial& d = dm[k];
    d = psrt::DevMaterial{};
    for (int ch = 0; ch < 3; ++ch) d.albedo[ch] = m.albedo[ch];
    d.fuzz = m.fuzz < 1 ? m.fuzz : 1;  // metal(a, f): fuzz(f < 1 ? f : 1)
    d.ir = m.ir;
    d.kind = m.kind;
  }
  HIP_TRY(hipSetDevice(c->device));
  {  // the last render may still read the materials
    const int rc = quiesce(c);
    if (rc) return rc;
  }
  if (n > c->mats_cap) {
    (void)hipFree(c->d_mats);
    c->d_mats = nullptr;
    c->mats_cap = 0;
    HIP_TRY(hipMalloc(&c->d_mats, (size_t)n * sizeof(psrt::DevMaterial)));
    c->mats_cap = n;
  }
  if (n > 0) {
    HIP_TRY(hipMemcpyAsync(c->d_mats, dm.data(), (size_t)n * sizeof(psrt::DevMaterial),
                           hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
  }
  c->lcam = *cam;
  c->mat_plist_valid = false;
  c->has_mats = true;
  return RT_OK;
}

int rt_render_materials(const rt_sphere* sph, const rt_material* mats, int n,
                        const rt_camera_lens* cam, const rt_params* p, double* accum_rgb,
                        unsigned char* rgb8, rt_stats* stats) {
  if (!cam || !p || !mats || n < 0 || (n > 0 && !sph))
    return set_error(RT_E_INVALID, "rt_render_materials: bad arguments");
  rt_params q = *p;
  q.flags |= RT_FLAG_MATERIALS;
  int rc = check_params(&q);
  if (rc) return rc;
  if (!accum_rgb && !rgb8 && rt_rows_owned(q.height, q.row_offset, q.row_stride) > 0)
    return set_error(RT_E_INVALID, "rt_render_materials: no output buffer");
  rt_context* c = nullptr;
  std::unique_lock<std::mutex> lk;
  rc = get_default_context(&c, &lk);
  if (rc) return rc;
  rc = rt_context_set_scene(c, sph, n, &cam->base);
  if (rc) return rc;
  rc = rt_context_set_materials(c, mats, n, cam);
  if (rc) return rc;
  return render_to_host(c, &q, accum_rgb, rgb8, stats);
}

// Debug entry: run one f64 primitive on the device (numerics parity tests).
int rt_debug_fail_after_trace(rt_context* c, int chunk) {
  if (!c) return set_error(RT_E_INVALID, "rt_debug_fail_after_trace: ctx is NULL");
  c->fail_after = chunk < 0 ? -1 : chunk;
  return RT_OK;
}

int rt_context_set_tuning(rt_context* c, const char* name, double value) {
  if (!name) return set_error(RT_E_INVALID, "rt_context_set_tuning: name is NULL");
  for (const TuningKey& k : kTuningKeys) {
    if (std::strcmp(k.name, name) != 0) continue;
    if (!std::isfinite(value))
      return set_error(RT_E_INVALID, "rt_context_set_tuning: %s must be finite", name);
    if (value < k.lo || value > k.hi)
      return set_error(RT_E_INVALID, "rt_context_set_tuning: %s = %g outside [%g, %g]", name, value,
                       k.lo, k.hi);
    if (c) {
      c->tune.*k.field = value;
    } else {
      std::lock_guard<std::mutex> lk(g_tuning_mu);
      g_tuning.*k.field = value;
    }
    return RT_OK;
  }
  return set_error(RT_E_INVALID, "rt_context_set_tuning: unknown knob '%s'", name);
}

int rt_context_get_tuning(rt_context* c, const char* name, double* value) {
  if (!name || !value) return set_error(RT_E_INVALID, "rt_context_get_tuning: bad arguments");
  const psrt::Tuning t = c ? c->tune : tuning_defaults();
  for (const TuningKey& k : kTuningKeys) {
    if (std::strcmp(k.name, name) != 0) continue;
    *value = t.*k.field;
    return RT_OK;
  }
  return set_error(RT_E_INVALID, "rt_context_get_tuning: unknown knob '%s'", name);
}

int rt_debug_probe_f64(int op, const double* x, const double* y, double* out, int n) {
  if (!x || !y || !out || n < 0) return set_error(RT_E_INVALID, "rt_debug_probe_f64: bad arguments");
  if (n == 0) return RT_OK;
  rt_context* c = nullptr;
  std::unique_lock<std::mutex> lk;
  int rc = get_default_context(&c, &lk);
  if (rc) return rc;
  ScratchBuf dx(c->stream), dy(c->stream), dout(c->stream);
  HIP_TRY(hipMalloc(&dx.p, n * sizeof(double)));
  HIP_TRY(hipMalloc(&dy.p, n * sizeof(double)));
  HIP_TRY(hipMalloc(&dout.p, n * sizeof(double)));
  // every copy on the context's stream: it is non-blocking, so null-stream
  // copies and memsets would not be ordered before the launch
  HIP_TRY(hipMemcpyAsync(dx.p, x, n * sizeof(double), hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(dy.p, y, n * sizeof(double), hipMemcpyHostToDevice, c->stream));
  hipLaunchKernelGGL(psrt::psrt_probe_f64, dim3((n + 255) / 256), dim3(256), 0, c->stream, op,
                     dx.as<const double>(), dy.as<const double>(), dout.as<double>(), (unsigned)n);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(out, dout.p, n * sizeof(double), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return RT_OK;
}

// Debug entry: hittable_list::hit on the device for `count` rays
// (rays[k] = {o, d, tmin, tmax}; out[k] = {index, p, normal, t, front_face});
// hints[k] (optional): the sphere ray k starts on, tested first as the trace
// kernel tests its previous hit (the neighbour-list and direction-map paths).
int rt_debug_world_hit_hint(const rt_sphere* sph, int n, const double* rays, const int* hints,
                            int count, double* out, int cull) {
  if (!rays || !out || count < 0 || n < 0 || (n > 0 && !sph))
    return set_error(RT_E_INVALID, "rt_debug_world_hit: bad arguments");
  if (count == 0) return RT_OK;
  rt_context* c = nullptr;
  std::unique_lock<std::mutex> lk;
  int rc = get_default_context(&c, &lk);
  if (rc) return rc;
  rt_camera cam{};
  rc = rt_context_set_scene(c, sph, n, &cam);
  if (rc) return rc;
  ScratchBuf dr(c->stream), dout(c->stream), dh(c->stream);
  HIP_TRY(hipMalloc(&dr.p, (size_t)count * 8 * sizeof(double)));
  HIP_TRY(hipMalloc(&dout.p, (size_t)count * 9 * sizeof(double)));
  // every copy and the memset on the context's stream: it is non-blocking, so
  // null-stream work would not be ordered before the launch (a null-stream
  // memset of dout once raced with the kernel and zeroed part of its output)
  HIP_TRY(hipMemcpyAsync(dr.p, rays, (size_t)count * 8 * sizeof(double), hipMemcpyHostToDevice,
                         c->stream));
  HIP_TRY(hipMemsetAsync(dout.p, 0, (size_t)count * 9 * sizeof(double), c->stream));
  if (hints) {
    HIP_TRY(hipMalloc(&dh.p, (size_t)count * sizeof(int)));
    HIP_TRY(hipMemcpyAsync(dh.p, hints, (size_t)count * sizeof(int), hipMemcpyHostToDevice,
                           c->stream));
  }
  hipLaunchKernelGGL(psrt::psrt_probe_hit, dim3((count + 63) / 64), dim3(64), 0, c->stream,
                     (const double4*)c->d_geo, (const double*)c->d_inv_r, n, dr.as<const double>(),
                     dh.as<const int>(), dout.as<double>(), (unsigned)count, bvh_view(c),
                     (cull && c->bvh) ? 1 : 0);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(out, dout.p, (size_t)count * 9 * sizeof(double), hipMemcpyDeviceToHost,
                         c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return RT_OK;
}

int rt_debug_world_hit(const rt_sphere* sph, int n, const double* rays, int count, double* out,
                       int cull) {
  return rt_debug_world_hit_hint(sph, n, rays, nullptr, count, out, cull);
}

}  // extern "C"
