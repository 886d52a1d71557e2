/*
 * rt.h — C ABI of the MI355X path-tracing hot path (libpsrt.so).
 *
 * This is the drop-in boundary for the reference's per-pixel loop. The
 * reference (fengye/PeterShirleyRaytracer) has no FFI: its hot path is the
 * pixel loop in main() (programs/main.cc:72-88), which calls
 * ray_color (programs/main.cc:34-49) -> hittable_list::hit
 * (programs/hittable_list.cc:3-20) -> sphere::hit (programs/sphere.cc:3-40)
 * -> vec3::random_in_hemisphere (programs/vec3.h:102-109), and quantises each
 * pixel with write_color (programs/color.h:8-24). Every entry point below
 * names the reference code it replaces.
 *
 * Conventions
 *   - 0 = success, negative = error (RT_E_*); rt_last_error() returns a
 *     thread-local message for the last failing call on this thread.
 *   - Plain pointers and sizes only. "host" buffers are caller-owned host
 *     memory; "device" buffers are caller-owned HIP device allocations on the
 *     context's device; "stream" is a hipStream_t passed as void* (NULL = the
 *     context's own stream).
 *   - Pixel order is the reference's output order (main.cc:72-75): output row
 *     r = 0 is the TOP row (reference j = H-1), columns i = 0..W-1 left to
 *     right. A shard owns rows r = row_offset + k*row_stride, k = 0,1,...
 *   - Threads and streams. rt_render and the rt_debug_* entries may be
 *     called from any number of host threads: they share the device's
 *     default context and hold a per-device lock for the whole call. An
 *     rt_context is used by one host thread at a time. Its renders may go to
 *     different streams: they share the context's device buffers, so the
 *     library orders them (a render on a new stream waits for the previous
 *     render on the device; rt_context_set_scene and buffer growth wait for it
 *     on the host). Frames meant to overlap use one context each.
 *   - Arithmetic is IEEE binary64 in the reference's operation order, no FMA
 *     contraction: accumulators are bit-identical to the reference's
 *     pixel_color (main.cc:77-84) for the same RNG stream.
 */
#ifndef PSRT_RT_H
#define PSRT_RT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RT_ABI_VERSION 7

/* ---- error codes ---------------------------------------------------------- */
#define RT_OK 0
#define RT_E_INVALID (-1)  /* bad argument (null pointer, size, shard)          */
#define RT_E_HIP (-2)      /* HIP runtime failure (message names the hipError) */
#define RT_E_NODEVICE (-3) /* no HIP device visible                            */
#define RT_E_NOMEM (-4)    /* device allocation failed                          */
#define RT_E_SCENE (-5)    /* scene not set / non-sphere object / too large     */

/* ---- scene ---------------------------------------------------------------- */

/* One flattened `sphere` (sphere.h:18-19: point3 centre; double radius).
 * hittable_list order is preserved: index k is objects[k]
 * (hittable_list.h:40), which decides ties (hittable_list.cc:11-15). */
typedef struct {
  double cx, cy, cz, r;
} rt_sphere;

/* The camera's public members (camera.h:31-35). get_ray(u,v) is
 * ray(origin, ((lower_left + horizontal*u) + vertical*v) - origin)
 * (camera.h:25-28). */
typedef struct {
  double origin[3];
  double lower_left[3];
  double horizontal[3];
  double vertical[3];
} rt_camera;

/* ---- render parameters ----------------------------------------------------- */

/* RNG streams. The reference draws from glibc rand() serially
 * (random.h:4-14), which no parallel device can reproduce; the device path
 * uses the COUNTER stream: one xorshift32 + Weyl stream per (pixel, sample)
 * (PCG32 until r05), fed through the reference's own random_double() mapping.
 * See DESIGN.md §RNG. */
#define RT_RNG_COUNTER 0

/* flags */
#define RT_FLAG_NONE 0
#define RT_FLAG_NO_CULL 1u /* force the linear sphere sweep (no BVH): same bits, slower */
#define RT_FLAG_NO_FIXPOINT 2u /* trace provably trapped paths to max_depth: same bits, slower */
/* scheduling hint, same bits: the launch's draining waves do not take issue
 * priority over other work (e.g. the next frame's launch on another stream) */
#define RT_FLAG_NO_TAIL_PRIORITY 4u
/* count the tests the device runs, by kind (rt_stats.tests_executed,
 * prerejects, box_tests, root_box_tests), with a slower kernel variant (~1%);
 * without it they read 0. Same bits; every other counter is always exact. */
#define RT_FLAG_CULL_STATS 8u
/* render with the material integrator and lens camera of the context
 * (rt_context_set_materials) instead of the reference's
 * diffuse ray_color */
#define RT_FLAG_MATERIALS 16u

typedef struct {
  int width;      /* image_width  (main.cc:57)                              */
  int height;     /* image_height (main.cc:58)                              */
  int spp;        /* sample_per_pixel (main.cc:66)                          */
  int max_depth;  /* max_depth (main.cc:68); up to max_depth+1 traced rays  */
  uint64_t seed;  /* counter-RNG seed                                       */
  int row_offset; /* first owned output row (0 = top)                       */
  int row_stride; /* owned rows are row_offset + k*row_stride (>= 1)        */
  unsigned flags; /* RT_FLAG_*                                              */
} rt_params;

/* Counters of one render (all ranks' shards add up to the frame's). */
typedef struct {
  uint64_t samples;        /* camera samples traced                          */
  uint64_t rays;           /* ray_color() invocations that called world.hit  */
  uint64_t sphere_tests;   /* sphere::hit calls of the reference = rays * n  */
  uint64_t tests_executed; /* sphere tests the device ran in full, in FP64
                              (sphere.cc:6-31); 0 without RT_FLAG_CULL_STATS */
  uint64_t box_tests;      /* FP32 BVH slab tests the device evaluated (same) */
  double kernel_ms;        /* device time of the trace kernels (HIP events)  */
  double total_ms;         /* device time of the whole render                */
  uint64_t rays_traced;    /* of `rays`, those the device traced; the rest
                              are the rays of provably trapped paths, ended
                              early with the same result     */
  uint64_t prerejects;     /* sphere candidates an exact FP32 pre-reject
                              decided without the FP64 test (same flag)     */
  uint64_t root_box_tests; /* FP64 ray / root-box tests of far origins (same) */
} rt_stats;

/* Number of rows a shard owns. */
int rt_rows_owned(int height, int row_offset, int row_stride);

/* ---- one-shot API (host buffers) ------------------------------------------ */

/* Replaces main.cc:72-88 for the owned rows: traces spp samples per pixel and
 * writes the FP64 pixel_color sums (rows_owned x width x 3, reference pixel
 * order) into accum_rgb (host) and, if rgb8 != NULL, the write_color bytes
 * (rows_owned x width x 3) into rgb8 (host). stats may be NULL.
 * Uses device 0 (or RT_DEVICE env). */
int rt_render(const rt_sphere* spheres, int n_spheres, const rt_camera* cam,
              const rt_params* params, double* accum_rgb, unsigned char* rgb8,
              rt_stats* stats);

/* Page-locked host memory for frame outputs (ABI 6). rt_render,
 * rt_render_materials and rt_group_render recognise it: psrt_reduce then
 * writes the sums and bytes straight into it across the link, with no
 * device-to-host copy and no pageable staging (DESIGN.md §7 "Host buffers").
 * Pinning is slow: allocate once and reuse across frames. Portable: usable
 * by every device. RT_E_NOMEM if the pages cannot be locked. */
int rt_host_alloc(size_t bytes, void** out);
int rt_host_free(void* p);
/* Page-lock existing host memory (e.g. a frame in POSIX shared memory that
 * several processes render into), with the same effect as rt_host_alloc
 * memory; rt_host_unregister before the memory is freed or unmapped. */
int rt_host_register(void* p, size_t bytes);
int rt_host_unregister(void* p);

/* write_color (color.h:8-24) on host data: (int)(255.999*clamp(sqrt(c*(1/spp)),0,0.999)). */
int rt_quantize_ppm(const double* accum_rgb, int width, int rows, int spp,
                    unsigned char* rgb8);

/* ---- context API (device-resident buffers, async) ------------------------- */

typedef struct rt_context rt_context;

int rt_context_create(int device, rt_context** out);
int rt_context_destroy(rt_context* ctx);

/* Flattened hittable_list + camera -> device constant buffers. */
int rt_context_set_scene(rt_context* ctx, const rt_sphere* spheres,
                         int n_spheres, const rt_camera* cam);

/* Output layout of the context's renders (ABI 6): consecutive rows of the
 * shard land accum_pitch doubles / rgb8_pitch bytes apart (0 = packed,
 * width * 3). With pitch G * width * 3 and the outputs pointing at row r of a
 * full frame, the G shards r = 0..G-1 (row_offset r, row_stride G) assemble one
 * frame in place: e.g. in page-locked host memory shared by G processes, with
 * no gather. Not with RT_FLAG_MATERIALS. */
int rt_context_set_row_pitch(rt_context* ctx, size_t accum_pitch, size_t rgb8_pitch);

/* Frames in flight (ABI 7): enqueue on `stream` a wait until ctx's last
 * enqueued trace launch has emptied its work queue (its first wave found no
 * more work: the launch's tail begins). A render enqueued on `stream` next,
 * with another context, then starts while ctx's last waves drain and takes
 * the CU slots their workgroups release, instead of sharing the GPU with
 * ctx's launch from its start or waiting for its end (bench.py frames in
 * flight). The wait holds however late it is enqueued: the
 * launch stores its number (counted per context, never reset) in a flag.
 * No-op before ctx's first render; RT_E_HIP if the device offers no signal
 * memory to wait on. ctx must outlive the wait: destroy it only after
 * `stream` has passed it (e.g. after synchronising `stream`). */
int rt_context_wait_drain(const rt_context* ctx, void* stream);

/* Enqueue a render of the owned rows on `stream` (after the context's
 * previous render, whatever its stream). A shard that owns no rows
 * (row_offset >= height) enqueues nothing and reports zero counters. d_accum (device,
 * rows_owned*width*3 doubles) and d_rgb8 (device, rows_owned*width*3 bytes)
 * may each be NULL. Returns after enqueueing; synchronise the stream before
 * reading. rt_context_sync_stats() reports the finished call's counters. */
int rt_render_device(rt_context* ctx, const rt_params* params, double* d_accum,
                     unsigned char* d_rgb8, void* stream);

/* Enqueue nframes (1..32) renders of the owned rows in one trace launch per
 * sample chunk: frame f is the frame of seed params->seed + f (the same
 * scene, camera and shard; bit-identical to rt_render_device with that
 * seed) and writes d_accum[f] / d_rgb8[f] (arrays of nframes device pointers,
 * either array or any entry may be NULL). The launch's tail (the last waves'
 * paths) is paid once per batch instead of once per frame.
 * rt_context_sync_stats() reports the batch's totals. rt_render_device is
 * this call with nframes = 1. */
int rt_render_device_frames(rt_context* ctx, const rt_params* params, int nframes,
                            double* const* d_accum, unsigned char* const* d_rgb8,
                            void* stream);

/* The context's own stream (hipStream_t as void*, non-blocking), used when
 * rt_render_device gets stream == NULL. One context per frame in flight
 * gives each frame its own stream (bench.py frame pipelining). */
void* rt_context_stream(rt_context* ctx);

/* Wait for the context's last render and fill stats (counters + kernel_ms).
 * Before the context's first render it fills zero counters and returns RT_OK.
 * After a render that failed part-way it waits for the part that was enqueued;
 * its counters are then not meaningful. */
int rt_context_sync_stats(rt_context* ctx, rt_stats* stats);

/* Device-side write_color over d_accum (rows*width*3) -> d_rgb8. */
int rt_quantize_device(rt_context* ctx, const double* d_accum, int width,
                       int rows, int spp, unsigned char* d_rgb8, void* stream);

/* ---- several devices, natively (psrt_group.cpp) -----------
 * One frame over a group of devices with no collective library: member g of
 * a G-member group renders the rows row_offset + (g + k*G)*row_stride of the
 * caller's shard on its own rt_context from its own host thread (interleaved
 * rows keep the load balanced), and copies them straight into their places in
 * the caller's host buffers: reference pixel order, bit-identical for every
 * G. Members may name the same device (each has its own context). This is the
 * C / C++ drop-in's multi-GPU path (one host thread per device); bench.py's is
 * one process per GPU over RCCL. RT_FLAG_MATERIALS is not supported here. */
typedef struct rt_group rt_group;
int rt_group_create(const int* devices, int n_devices, rt_group** out);
int rt_group_destroy(rt_group* group);
int rt_group_size(const rt_group* group);
/* member's context (tuning knobs, stats), or NULL when out of range */
rt_context* rt_group_context(rt_group* group, int member);
int rt_group_set_scene(rt_group* group, const rt_sphere* spheres, int n_spheres,
                       const rt_camera* cam);
/* accum_rgb / rgb8: host, rows_owned(params) x width x 3 (either may be NULL);
 * stats: counts summed over members, kernel_ms / total_ms the slowest member's */
int rt_group_render(rt_group* group, const rt_params* params, double* accum_rgb,
                    unsigned char* rgb8, rt_stats* stats);
/* One-shot: rt_group_create + set_scene + render + destroy. */
int rt_render_devices(const rt_sphere* spheres, int n_spheres, const rt_camera* cam,
                      const rt_params* params, const int* devices, int n_devices,
                      double* accum_rgb, unsigned char* rgb8, rt_stats* stats);

/* ---- scene helpers (host) -------------------------------------------------- */

/* camera() default constructor (camera.h:11-23): 16:9, viewport 2 high,
 * focal length 1, origin 0. */
int rt_camera_default(rt_camera* out);

/* lookfrom/lookat pinhole (extension; no defocus): the book's
 * camera(lookfrom, lookat, vup, vfov_degrees, aspect). */
int rt_camera_look_at(const double lookfrom[3], const double lookat[3],
                      const double vup[3], double vfov_deg, double aspect,
                      rt_camera* out);

/* The reference's two-sphere world (main.cc:61-63). Returns the count (2);
 * writes at most cap records. */
int rt_scene_two_spheres(rt_sphere* out, int cap);

/* The final random-spheres scene: glibc srand(seed)
 * stream, ground r=1000, 22x22 jittered r=0.2 grid, three r=1 spheres,
 * diffuse-only. Returns the sphere count; writes at most cap records. */
int rt_scene_random_spheres(unsigned int seed, rt_sphere* out, int cap);

/* ---- materials and defocus (extension: SURVEY.md §8(f)4; parity unpinned) ---
 * The reference traces one material, 0.5-attenuation hemisphere diffuse
 * (main.cc:42-43), through a fixed pinhole (camera.h:11-23). The book it
 * follows (Ray Tracing in One Weekend v3.2, ch. 9-13) goes on to materials
 * and a thin-lens camera; this is that integrator, restated:
 *   ray_color: depth <= 0 -> black; world.hit(r, 0.001, inf); on a hit the
 *     material scatters (attenuation * ray_color(scattered, depth - 1), the
 *     product taken innermost first, as the recursion does) or absorbs
 *     (black); a miss returns the sky of main.cc:46-48.
 *   lambertian: normal + random_unit_vector() (vec3.h:97-100), the normal when
 *     that is near zero (all |e| < 1e-8); metal: reflect(unit(d), n) +
 *     fuzz * random_in_unit_sphere(), absorbed unless dot(scattered, n) > 0;
 *   dielectric: Snell / Schlick (pow(x, 5) evaluated as (x*x)*(x*x)*x), one
 *     random_double() drawn only when refraction is possible.
 *   thin lens: get_ray(s, t) offsets the origin by lens_radius *
 *     random_in_unit_disk() (g++ draw order: y then x) along u, v.
 * No reference output exists for any of this: tests check the device
 * against a CPU restatement of it bit for bit ("parity unpinned"). */
#define RT_MAT_LAMBERTIAN 0
#define RT_MAT_METAL 1
#define RT_MAT_DIELECTRIC 2

/* One material per sphere, same index as the sphere list. */
typedef struct {
  int kind;          /* RT_MAT_*                                      */
  int reserved;      /* 0                                             */
  double albedo[3];  /* lambertian / metal attenuation                */
  double fuzz;       /* metal: reflection fuzz (book clamps to <= 1)  */
  double ir;         /* dielectric: index of refraction               */
} rt_material;

/* The thin-lens camera: the pinhole basis plus the lens frame. */
typedef struct {
  rt_camera base;     /* origin, lower_left, horizontal, vertical (focus plane) */
  double u[3], v[3];  /* unit lens axes (camera right / up)                     */
  double lens_radius; /* aperture / 2; the disk is always sampled (the book's
                         stream), radius 0 only zeroes the offset, so an
                         aperture-0 camera draws differently from rt_render */
} rt_camera_lens;

/* camera(lookfrom, lookat, vup, vfov, aspect, aperture, focus_dist) of the
 * book (ch. 12); with aperture 0 and focus_dist 1 its base equals
 * rt_camera_look_at. */
int rt_camera_look_at_lens(const double lookfrom[3], const double lookat[3],
                           const double vup[3], double vfov_deg, double aspect,
                           double aperture, double focus_dist, rt_camera_lens* out);

/* The book's random_scene() (ch. 13) on the glibc srand(seed) stream, with
 * g++'s argument evaluation order for every vec3 built from draws: ground
 * (lambertian 0.5), 22x22 jittered r = 0.2 spheres (80% lambertian with
 * albedo random()*random(), 15% metal, 5% glass 1.5), glass / lambertian /
 * metal r = 1 spheres. Returns the sphere count; writes at most cap records
 * into out and mats (either may be NULL). */
int rt_scene_book_final(unsigned int seed, rt_sphere* out, rt_material* mats, int cap);

/* Materials (one per sphere of the context's scene, same order) and the lens
 * camera for renders with RT_FLAG_MATERIALS. n must equal the scene's count.
 * mats == NULL clears them. */
int rt_context_set_materials(rt_context* ctx, const rt_material* mats, int n,
                             const rt_camera_lens* cam);

/* One-shot material render (rt_render with RT_FLAG_MATERIALS): host buffers. */
int rt_render_materials(const rt_sphere* spheres, const rt_material* mats, int n_spheres,
                        const rt_camera_lens* cam, const rt_params* params,
                        double* accum_rgb, unsigned char* rgb8, rt_stats* stats);

/* ---- scene files (extension: SURVEY.md §8(f)3) ------------------------------
 * Text form of main.cc:53-63 (spheres in hittable_list order, camera,
 * pixel-loop parameters); grammar in psrt_scenefile.cpp and DESIGN.md
 * §Scene files. Decimal or hex-float numbers; %.17g output round-trips.
 *
 * rt_scene_parse / rt_scene_load: returns the sphere count (writes at most
 * cap records; call again with a larger buffer if it exceeds cap) or
 * RT_E_SCENE / RT_E_INVALID. cam (optional) receives the file's camera, or
 * camera() when it has none. params (optional): only the fields the file's
 * `render` line names are overwritten (width, height, spp, max_depth, seed);
 * `aspect auto` uses width/height from the file, else from *params. */
int rt_scene_parse(const char* text, rt_sphere* out, int cap, rt_camera* cam,
                   rt_params* params);
int rt_scene_load(const char* path, rt_sphere* out, int cap, rt_camera* cam,
                  rt_params* params);

/* Writes the scene file text (camera as a basis, `render` line only when
 * params != NULL) into buf (NUL-terminated, truncated to cap-1 chars).
 * Returns the full text length (snprintf-style) or a negative error. */
long long rt_scene_format(const rt_sphere* spheres, int n_spheres, const rt_camera* cam,
                          const rt_params* params, char* buf, size_t cap);

/* ---- misc ----------------------------------------------------------------- */
const char* rt_last_error(void);
int rt_abi_version(void);
int rt_device_count(void);
const char* rt_build_info(void);

/* Debug: run one binary64 primitive on the device, element-wise
 * (op 0 sqrt(x), 1 x/y, 2 x*y, 3 x+y, 4 x*y+x uncontracted, 5 ldexp(x,(int)y),
 * 6 sqrt(x) as the trace kernel computes it).
 * Used by the numerics parity tests. */
int rt_debug_probe_f64(int op, const double* x, const double* y, double* out, int n);

/* Debug: hittable_list::hit (hittable_list.cc:3-20) on the device with the
 * megakernel's own code, one ray per thread. rays[k*8..] = {ox,oy,oz,dx,dy,dz,
 * tmin,tmax}; out[k*9..] = {index (-1 miss), px,py,pz, nx,ny,nz, t, front_face}.
 * cull != 0: rays with tmin == 0 and tmax == +inf (the trace kernel's call)
 * go through the BVH path when the scene has one. */
int rt_debug_world_hit(const rt_sphere* spheres, int n_spheres, const double* rays,
                       int count, double* out, int cull);

/* Debug: as rt_debug_world_hit, with hints[k] (NULL = none; -1 = none for ray
 * k) naming the sphere ray k starts on. The trace kernel tests a bounce ray's
 * previous hit first and, when that hit is close to the ray's origin, takes
 * that sphere's neighbour list as hit_quick's candidate list;
 * the record is the reference's whatever the hint. */
int rt_debug_world_hit_hint(const rt_sphere* spheres, int n_spheres, const double* rays,
                            const int* hints, int count, double* out, int cull);

/* ---- tuning (measurement and tests only) ------------------------------------
 * The render path reads no environment variable. These knobs exist for A/B
 * measurements and for tests that force a code path; every one keeps the
 * output bit-identical (only the sample-buffer cap and the diagnostic variant
 * change anything but time: chunking, and the stamps on stderr).
 *   sample_buf_mb   cap of the sample-record buffer, MiB (default 49152)
 *   queue_k, queue_d  guided work-queue shape (2, 2; psrt_capi.hip queue_phases)
 *   linear_chunk    queue ticket of the small-scene path (0: 1024)
 *   no_camlist, no_neighbors, no_fixpoint, no_lds  1 disables that exact shortcut
 *   blocks_per_cu   cap on resident trace workgroups per CU (0: occupancy max)
 *   mat_lds         material kernel's scene in LDS: -1 auto, 0 off, 1 on
 *   mat_batch       parked lanes per batched walk of the material kernel (48)
 *   flush_at        per-lane counter flush threshold (0: computed)
 *   stamps          1: the diagnostic kernel variant (section clocks on stderr)
 *   scene_rebuild   1: rebuild the culling structures for an unchanged scene
 *   big_ratio       radius ratio of the big-sphere class (0: 16)
 *   reduce_lean     1: psrt_reduce_lean, which fits beside a resident trace
 *                   launch (frames in flight; max_depth <= 1000 only)
 * ctx == NULL sets / reads the process defaults: a context copies them at
 * rt_context_create, the one-shot entries' default contexts at every call.
 * Unknown names and non-finite values fail with RT_E_INVALID. */
int rt_context_set_tuning(rt_context* ctx, const char* name, double value);
int rt_context_get_tuning(rt_context* ctx, const char* name, double* value);

/* Debug (fault injection, tests only): the context's NEXT render fails with
 * RT_E_HIP after sample chunk `chunk`'s trace launch and before its reduce, as
 * a HIP error there would (the reference and the material integrator alike);
 * the hook then clears itself. chunk < 0 clears it.
 * The failure-recovery path (queue heads and counter sets re-zeroed by the
 * next render) is tested through it. */
int rt_debug_fail_after_trace(rt_context* ctx, int chunk);

#ifdef __cplusplus
}
#endif

#endif /* PSRT_RT_H */
