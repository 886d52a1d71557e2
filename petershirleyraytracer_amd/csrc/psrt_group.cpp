// psrt_group.cpp — one frame over several devices, natively (no torch, no
// collective library): the C ABI's device group (include/rt.h rt_group_*).
//
// The reference's pixel loop (main.cc:72-88) is embarrassingly parallel over
// pixels once every (pixel, sample) has its own counter stream,
// so a frame shards over devices with no exchange but the framebuffer: member
// g of a G-member group renders the rows row_offset + (g + kG) row_stride of
// the caller's shard (interleaved rows: contiguous bands are 0.15-1.32x the
// mean cost on the final scene) on its own rt_context, from its
// own host thread, and copies its rows straight into their places in the
// caller's buffer (a strided 2-D copy): the gather into reference pixel
// order is the copies themselves. A pixel's sum never leaves its lane, so the
// frame is bit-identical for every G (tests/test_gpu_group.py).
//
// Members may share a device (a test renders G = 2, 3, 8 members on one GPU);
// each member owns its context, stream and device buffers.
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <climits>
#include <cstring>
#include <exception>
#include <string>
#include <thread>
#include <vector>

#include "../../include/rt.h"
#include "psrt_error.h"

namespace {

struct Member {
  int device = 0;
  rt_context* ctx = nullptr;
  double* d_accum = nullptr;  // this member's rows, contiguous
  unsigned char* d_rgb = nullptr;
  size_t cap = 0;  // pixels the buffers hold
};

// The device address of page-locked host memory (rt_host_alloc /
// rt_host_register), or nullptr for pageable memory.
void* mapped_host(const void* p) {
  if (!p) return nullptr;
  hipPointerAttribute_t at{};
  if (hipPointerGetAttributes(&at, p) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  return at.type == hipMemoryTypeHost ? at.devicePointer : nullptr;
}

int hip_err(hipError_t e, const char* what) {
  return psrt::set_error(e == hipErrorOutOfMemory ? RT_E_NOMEM : RT_E_HIP, "%s: %s", what,
                         hipGetErrorString(e));
}

}  // namespace

struct rt_group {
  std::vector<Member> m;
};

namespace {

// One member's share of a render: its sub-shard of the caller's rows on its
// context, then its rows into the caller's host buffers at stride G rows.
int member_render(Member& mb, int g, int G, const rt_params& p, double* accum,
                  unsigned char* rgb8, rt_stats* st) {
  rt_params q = p;
  q.row_offset = p.row_offset + g * p.row_stride;  // rows row_offset + (g + kG) row_stride
  q.row_stride = p.row_stride * G;
  *st = rt_stats{};
  const int rows = rt_rows_owned(q.height, q.row_offset, q.row_stride);
  if (rows <= 0) return RT_OK;  // more members than rows: this one owns none
  const size_t P = (size_t)rows * q.width;
  hipError_t e = hipSetDevice(mb.device);
  if (e != hipSuccess) return hip_err(e, "hipSetDevice");
  const size_t W3 = (size_t)q.width * 3;
  // Page-locked caller buffers (rt_host_alloc): the member's reduce writes its
  // rows straight into their places, G rows apart (rt_context_set_row_pitch),
  // with no device buffers and no copy
  double* h_acc = (double*)mapped_host(accum);
  unsigned char* h_rgb = (unsigned char*)mapped_host(rgb8);
  if (accum && h_acc && (!rgb8 || h_rgb)) {
    int rc = rt_context_set_row_pitch(mb.ctx, (size_t)G * W3, (size_t)G * W3);
    if (rc) return rc;
    rc = rt_render_device(mb.ctx, &q, h_acc + (size_t)g * W3, rgb8 ? h_rgb + (size_t)g * W3 : nullptr,
                          nullptr);
    if (!rc) rc = rt_context_sync_stats(mb.ctx, st);  // waits for the render
    const int rc2 = rt_context_set_row_pitch(mb.ctx, 0, 0);
    return rc ? rc : rc2;
  }
  if (mb.cap < P) {
    (void)hipFree(mb.d_accum);
    (void)hipFree(mb.d_rgb);
    mb.d_accum = nullptr;
    mb.d_rgb = nullptr;
    mb.cap = 0;
    if ((e = hipMalloc(&mb.d_accum, P * 3 * sizeof(double))) != hipSuccess)
      return hip_err(e, "hipMalloc");
    if ((e = hipMalloc(&mb.d_rgb, P * 3)) != hipSuccess) return hip_err(e, "hipMalloc");
    mb.cap = P;
  }
  int rc = rt_render_device(mb.ctx, &q, mb.d_accum, rgb8 ? mb.d_rgb : nullptr, nullptr);
  if (rc) return rc;
  hipStream_t s = (hipStream_t)rt_context_stream(mb.ctx);
  // Once a copy into the caller's buffers is enqueued, every return waits for
  // the stream: no copy may still write them after rt_group_render returns.
  auto fail = [&](int code) {
    (void)hipStreamSynchronize(s);
    return code;
  };
  // row k of this member is row g + kG of the caller's shard
  if (accum &&
      (e = hipMemcpy2DAsync(accum + (size_t)g * W3, (size_t)G * W3 * sizeof(double), mb.d_accum,
                            W3 * sizeof(double), W3 * sizeof(double), (size_t)rows,
                            hipMemcpyDeviceToHost, s)) != hipSuccess)
    return fail(hip_err(e, "hipMemcpy2DAsync"));
  if (rgb8 && (e = hipMemcpy2DAsync(rgb8 + (size_t)g * W3, (size_t)G * W3, mb.d_rgb, W3, W3,
                                    (size_t)rows, hipMemcpyDeviceToHost, s)) != hipSuccess)
    return fail(hip_err(e, "hipMemcpy2DAsync"));
  rc = rt_context_sync_stats(mb.ctx, st);  // waits for the render
  if (rc) return fail(rc);
  if ((e = hipStreamSynchronize(s)) != hipSuccess) return hip_err(e, "hipStreamSynchronize");
  return RT_OK;
}

}  // namespace

extern "C" {

int rt_group_create(const int* devices, int n, rt_group** out) {
  if (!out || !devices || n < 1 || n > 1024)
    return psrt::set_error(RT_E_INVALID, "rt_group_create: bad arguments");
  *out = nullptr;
  rt_group* grp = new rt_group();
  for (int g = 0; g < n; ++g) {
    Member mb;
    mb.device = devices[g];
    const int rc = rt_context_create(devices[g], &mb.ctx);
    if (rc) {
      rt_group_destroy(grp);
      return rc;
    }
    grp->m.push_back(mb);
  }
  *out = grp;
  return RT_OK;
}

int rt_group_destroy(rt_group* grp) {
  if (!grp) return RT_OK;
  for (Member& mb : grp->m) {
    if (!mb.ctx) continue;
    rt_context_destroy(mb.ctx);  // waits for the member's last render
    (void)hipSetDevice(mb.device);
    (void)hipFree(mb.d_accum);
    (void)hipFree(mb.d_rgb);
  }
  delete grp;
  return RT_OK;
}

int rt_group_size(const rt_group* grp) { return grp ? (int)grp->m.size() : 0; }

rt_context* rt_group_context(rt_group* grp, int member) {
  if (!grp || member < 0 || member >= (int)grp->m.size()) return nullptr;
  return grp->m[member].ctx;
}

int rt_group_set_scene(rt_group* grp, const rt_sphere* sph, int n, const rt_camera* cam) {
  if (!grp) return psrt::set_error(RT_E_INVALID, "rt_group_set_scene: group is NULL");
  // every member builds its culling structures (host BVH + uploads), in parallel
  std::vector<int> rc(grp->m.size(), RT_OK);
  std::vector<std::string> err(grp->m.size());
  std::vector<std::thread> th;
  th.reserve(grp->m.size());
  try {
    for (size_t g = 0; g < grp->m.size(); ++g)
      th.emplace_back([&, g] {
        rc[g] = rt_context_set_scene(grp->m[g].ctx, sph, n, cam);
        if (rc[g]) err[g] = rt_last_error();
      });
  } catch (const std::exception& e) {
    for (auto& t : th) t.join();
    return psrt::set_error(RT_E_NOMEM, "rt_group_set_scene: cannot start a member thread: %s",
                           e.what());
  }
  for (auto& t : th) t.join();
  for (size_t g = 0; g < rc.size(); ++g)
    if (rc[g]) return psrt::set_error(rc[g], "member %zu: %s", g, err[g].c_str());
  return RT_OK;
}

int rt_group_render(rt_group* grp, const rt_params* p, double* accum_rgb, unsigned char* rgb8,
                    rt_stats* stats) {
  if (!grp || !p) return psrt::set_error(RT_E_INVALID, "rt_group_render: bad arguments");
  // the members' own renders would check these too, but only after their
  // shard arithmetic and buffer sizing ran on the unchecked values
  int prc = psrt::check_render_params(p);
  if (prc) return prc;
  if (p->flags & RT_FLAG_MATERIALS)
    return psrt::set_error(RT_E_INVALID, "rt_group_render: RT_FLAG_MATERIALS is not supported");
  const int G = (int)grp->m.size();
  if ((long long)p->row_stride * G > INT_MAX ||
      (long long)p->row_offset + (long long)(G - 1) * p->row_stride > INT_MAX)
    return psrt::set_error(RT_E_INVALID, "rt_group_render: row_stride %d x %d members overflows",
                           p->row_stride, G);
  if (!accum_rgb && !rgb8 && rt_rows_owned(p->height, p->row_offset, p->row_stride) > 0)
    return psrt::set_error(RT_E_INVALID, "rt_group_render: no output buffer");
  std::vector<int> rc(G, RT_OK);
  std::vector<std::string> err(G);
  std::vector<rt_stats> st(G);
  std::vector<std::thread> th;
  th.reserve(G);
  try {
    for (int g = 0; g < G; ++g)
      th.emplace_back([&, g] {
        try {
          rc[g] = member_render(grp->m[g], g, G, *p, accum_rgb, rgb8, &st[g]);
        } catch (const std::exception& e) {
          rc[g] = psrt::set_error(RT_E_HIP, "%s", e.what());
        }
        if (rc[g]) err[g] = rt_last_error();
      });
  } catch (const std::exception& e) {  // std::system_error: no thread for a member
    for (auto& t : th) t.join();
    return psrt::set_error(RT_E_NOMEM, "rt_group_render: cannot start a member thread: %s",
                           e.what());
  }
  for (auto& t : th) t.join();
  for (int g = 0; g < G; ++g)
    if (rc[g]) return psrt::set_error(rc[g], "member %d: %s", g, err[g].c_str());
  if (stats) {
    rt_stats s{};
    for (const rt_stats& x : st) {  // counts add up; times are the slowest member's
      s.samples += x.samples;
      s.rays += x.rays;
      s.sphere_tests += x.sphere_tests;
      s.tests_executed += x.tests_executed;
      s.box_tests += x.box_tests;
      s.rays_traced += x.rays_traced;
      s.prerejects += x.prerejects;
      s.root_box_tests += x.root_box_tests;
      s.kernel_ms = std::max(s.kernel_ms, x.kernel_ms);
      s.total_ms = std::max(s.total_ms, x.total_ms);
    }
    *stats = s;
  }
  return RT_OK;
}

int rt_render_devices(const rt_sphere* sph, int n, const rt_camera* cam, const rt_params* p,
                      const int* devices, int n_devices, double* accum_rgb, unsigned char* rgb8,
                      rt_stats* stats) {
  rt_group* grp = nullptr;
  int rc = rt_group_create(devices, n_devices, &grp);
  if (rc) return rc;
  rc = rt_group_set_scene(grp, sph, n, cam);
  if (!rc) rc = rt_group_render(grp, p, accum_rgb, rgb8, stats);
  std::string keep = rc ? rt_last_error() : std::string();
  rt_group_destroy(grp);
  if (rc) return psrt::set_error(rc, "%s", keep.c_str());
  return RT_OK;
}

}  // extern "C"
