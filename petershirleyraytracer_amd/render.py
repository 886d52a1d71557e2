"""Host-side interface of the hot path (Python over the C ABI of include/rt.h).

Mirrors the reference's pieces by name and meaning:

* ``camera_default()``            camera() (camera.h:11-23)
* ``camera_look_at(...)``         look-at pinhole extension for the final scene
* ``scene_two_spheres()``         main.cc:61-63 world
* ``scene_random_spheres(seed)``  final random-spheres world
* ``load_scene / parse_scene``    scene/camera files (DESIGN.md §Scene files)
* ``save_scene / format_scene``   ... and back (bit-exact round trip)
* ``render(...)``                 the main.cc:72-88 pixel loop for a shard of rows
* ``render_materials(...)``       the book's material integrator + thin lens
                                  (extension; parity unpinned)
* ``write_ppm(...)``              main.cc:70 header + color.h:21-23 pixel lines

Scenes are ``(n, 4)`` float64 arrays of (cx, cy, cz, r) in hittable_list order;
cameras are ``(4, 3)`` float64 arrays (origin, lower_left, horizontal, vertical).
"""
from __future__ import annotations

import ctypes as C
import weakref
from contextlib import contextmanager
from dataclasses import dataclass
from typing import Optional

import numpy as np

from . import _lib
from ._lib import RtCamera, RtCameraLens, RtMaterial, RtParams, RtSphere, RtStats, check


def _spheres(spheres) -> tuple:
    arr = np.ascontiguousarray(np.asarray(spheres, dtype=np.float64).reshape(-1, 4))
    buf = (RtSphere * max(1, len(arr)))()
    if len(arr):
        C.memmove(buf, arr.ctypes.data, arr.nbytes)
    return buf, len(arr)


def _camera(cam) -> RtCamera:
    a = np.asarray(cam, dtype=np.float64).reshape(4, 3)
    c = RtCamera()
    for k in range(3):
        c.origin[k], c.lower_left[k] = a[0, k], a[1, k]
        c.horizontal[k], c.vertical[k] = a[2, k], a[3, k]
    return c


def _camera_array(c: RtCamera) -> np.ndarray:
    return np.array([list(c.origin), list(c.lower_left), list(c.horizontal),
                     list(c.vertical)], dtype=np.float64)


FLAG_NO_CULL = 1
FLAG_NO_FIXPOINT = 2  # trace provably trapped paths to max_depth (same bits, slower)
FLAG_NO_TAIL_PRIORITY = 4  # scheduling hint: no issue priority for the launch tail (same bits)
FLAG_CULL_STATS = 8  # count executed sphere / box tests (slower kernel variant; else they read 0)
FLAG_MATERIALS = 16  # the material integrator of the context (rt_context_set_materials)

# Materials are (n, 6) float64 rows (kind, albedo r, g, b, fuzz, ir), one per
# sphere in hittable_list order (include/rt.h rt_material).
MAT_LAMBERTIAN, MAT_METAL, MAT_DIELECTRIC = 0, 1, 2


def _materials(mats) -> tuple:
    a = np.asarray(mats, dtype=np.float64).reshape(-1, 6)
    buf = (RtMaterial * max(1, len(a)))()
    for k, row in enumerate(a):
        buf[k].kind = int(row[0])
        buf[k].albedo[0], buf[k].albedo[1], buf[k].albedo[2] = row[1], row[2], row[3]
        buf[k].fuzz, buf[k].ir = row[4], row[5]
    return buf, len(a)


def _materials_array(buf, n: int) -> np.ndarray:
    return np.array([[buf[k].kind, *list(buf[k].albedo), buf[k].fuzz, buf[k].ir]
                     for k in range(n)], dtype=np.float64).reshape(n, 6)


@dataclass
class LensCamera:
    """The book's thin-lens camera (rt_camera_lens): the focus-plane basis
    (4, 3) as camera arrays, the lens axes u, v and lens_radius."""
    base: np.ndarray
    u: np.ndarray
    v: np.ndarray
    lens_radius: float

    def to_c(self) -> RtCameraLens:
        c = RtCameraLens()
        c.base = _camera(self.base)
        for k in range(3):
            c.u[k], c.v[k] = float(self.u[k]), float(self.v[k])
        c.lens_radius = float(self.lens_radius)
        return c


def camera_look_at_lens(lookfrom=(13.0, 2.0, 3.0), lookat=(0.0, 0.0, 0.0), vup=(0.0, 1.0, 0.0),
                        vfov: float = 20.0, aspect: float = 1.5, aperture: float = 0.1,
                        focus_dist: float = 10.0) -> LensCamera:
    """camera(lookfrom, lookat, vup, vfov, aspect, aperture, focus_dist) (book ch. 12)."""
    c = RtCameraLens()
    d3 = C.c_double * 3
    check(_lib.load().rt_camera_look_at_lens(d3(*lookfrom), d3(*lookat), d3(*vup), vfov, aspect,
                                             aperture, focus_dist, C.byref(c)),
          "rt_camera_look_at_lens")
    return LensCamera(_camera_array(c.base), np.array(list(c.u)), np.array(list(c.v)),
                      c.lens_radius)


def scene_book_final(seed: int = 1):
    """The book's random_scene() with materials: (spheres (n, 4), materials (n, 6))."""
    L = _lib.load()
    n = L.rt_scene_book_final(seed, None, None, 0)
    sp = (RtSphere * n)()
    mt = (RtMaterial * n)()
    L.rt_scene_book_final(seed, sp, mt, n)
    return (np.frombuffer(sp, dtype=np.float64, count=4 * n).reshape(n, 4).copy(),
            _materials_array(mt, n))


def params(width: int, height: int, spp: int, max_depth: int = 50, seed: int = 0,
           row_offset: int = 0, row_stride: int = 1, flags: int = 0) -> RtParams:
    return RtParams(width, height, spp, max_depth, seed, row_offset, row_stride, flags)


def rows_owned(height: int, row_offset: int = 0, row_stride: int = 1) -> int:
    return _lib.load().rt_rows_owned(height, row_offset, row_stride)


def camera_default() -> np.ndarray:
    c = RtCamera()
    check(_lib.load().rt_camera_default(C.byref(c)), "rt_camera_default")
    return _camera_array(c)


def camera_look_at(lookfrom=(13.0, 2.0, 3.0), lookat=(0.0, 0.0, 0.0), vup=(0.0, 1.0, 0.0),
                   vfov: float = 20.0, aspect: float = 1.5) -> np.ndarray:
    c = RtCamera()
    d3 = C.c_double * 3
    check(_lib.load().rt_camera_look_at(d3(*lookfrom), d3(*lookat), d3(*vup), vfov, aspect,
                                        C.byref(c)), "rt_camera_look_at")
    return _camera_array(c)


def scene_two_spheres() -> np.ndarray:
    buf = (RtSphere * 2)()
    n = _lib.load().rt_scene_two_spheres(buf, 2)
    return np.frombuffer(buf, dtype=np.float64, count=4 * n).reshape(n, 4).copy()


def scene_random_spheres(seed: int = 1) -> np.ndarray:
    L = _lib.load()
    n = L.rt_scene_random_spheres(seed, None, 0)
    buf = (RtSphere * n)()
    L.rt_scene_random_spheres(seed, buf, n)
    return np.frombuffer(buf, dtype=np.float64, count=4 * n).reshape(n, 4).copy()


@dataclass
class SceneFile:
    """A parsed scene file: spheres (n, 4), camera (4, 3) and the pixel-loop
    parameters (0 / 50 / 0 where the file's ``render`` line is silent)."""
    spheres: np.ndarray
    camera: np.ndarray
    width: int = 0
    height: int = 0
    spp: int = 0
    max_depth: int = 50
    seed: int = 0


def _scene_call(fn, arg) -> SceneFile:
    L = _lib.load()
    cam = RtCamera()
    p = params(0, 0, 0)
    n = getattr(L, fn)(arg, None, 0, C.byref(cam), C.byref(p))
    check(min(n, 0), fn)
    buf = (RtSphere * max(1, n))()
    check(min(getattr(L, fn)(arg, buf, n, None, None), 0), fn)
    arr = np.frombuffer(buf, dtype=np.float64, count=4 * n).reshape(n, 4).copy()
    return SceneFile(arr, _camera_array(cam), p.width, p.height, p.spp, p.max_depth, p.seed)


def parse_scene(text: str) -> SceneFile:
    """rt_scene_parse over the text of a ``psrt-scene 1`` file."""
    return _scene_call("rt_scene_parse", text.encode())


def load_scene(path: str) -> SceneFile:
    """rt_scene_load: read a ``psrt-scene 1`` file."""
    return _scene_call("rt_scene_load", str(path).encode())


def format_scene(spheres, camera=None, width: Optional[int] = None, height: int = 0,
                 spp: int = 0, max_depth: int = 50, seed: int = 0) -> str:
    """rt_scene_format: the file text (``render`` line only when width is given)."""
    L = _lib.load()
    buf, n = _spheres(spheres)
    cam = C.byref(_camera(camera)) if camera is not None else None
    p = C.byref(params(width, height, spp, max_depth, seed)) if width is not None else None
    size = L.rt_scene_format(buf, n, cam, p, None, 0)
    check(int(min(size, 0)), "rt_scene_format")
    out = C.create_string_buffer(int(size) + 1)
    L.rt_scene_format(buf, n, cam, p, out, size + 1)
    return out.value.decode()


def save_scene(path: str, spheres, camera=None, **render_args) -> None:
    with open(path, "w") as f:
        f.write(format_scene(spheres, camera, **render_args))


def stats_dict(s: RtStats) -> dict:
    return dict(samples=s.samples, rays=s.rays, sphere_tests=s.sphere_tests,
                tests_executed=s.tests_executed, box_tests=s.box_tests,
                kernel_ms=s.kernel_ms, total_ms=s.total_ms, rays_traced=s.rays_traced,
                prerejects=s.prerejects, root_box_tests=s.root_box_tests)


def host_array(shape, dtype=np.float64) -> np.ndarray:
    """A numpy array in page-locked host memory (rt_host_alloc, include/rt.h):
    passed as a render's output (render(..., out=...)), the frame is written
    into it by the device across the link with no copy. Pinning is slow:
    allocate once, reuse across frames. Freed with the array."""
    L = _lib.load()
    dt = np.dtype(dtype)
    count = int(np.prod(shape)) if len(tuple(np.atleast_1d(shape))) else 1
    nbytes = max(1, count * dt.itemsize)
    ptr = C.c_void_p()
    check(L.rt_host_alloc(nbytes, C.byref(ptr)), "rt_host_alloc")
    buf = (C.c_ubyte * nbytes).from_address(ptr.value)
    arr = np.frombuffer(buf, dtype=np.uint8, count=count * dt.itemsize).view(dt).reshape(shape)
    weakref.finalize(buf, L.rt_host_free, C.c_void_p(ptr.value))
    return arr


def _out_arrays(out, rows: int, width: int, want_rgb: bool):
    """The caller's output arrays (out = (accum, rgb8 or None)), checked, or new ones."""
    if out is None:
        return (np.zeros((rows, width, 3), dtype=np.float64),
                np.zeros((rows, width, 3), dtype=np.uint8) if want_rgb else None)
    acc, rgb = out
    if acc is None and rgb is None:
        raise ValueError("out needs at least one array")
    if acc is not None and (acc.shape != (rows, width, 3) or acc.dtype != np.float64
                            or not acc.flags.c_contiguous):
        raise ValueError(f"out accum must be C-contiguous float64 {(rows, width, 3)}")
    if rgb is not None and (rgb.shape != (rows, width, 3) or rgb.dtype != np.uint8
                            or not rgb.flags.c_contiguous):
        raise ValueError(f"out rgb8 must be C-contiguous uint8 {(rows, width, 3)}")
    if (acc is not None and not acc.flags.writeable) or (rgb is not None and not rgb.flags.writeable):
        raise ValueError("out arrays must be writeable")
    return acc, rgb


def render(spheres, camera, width: int, height: int, spp: int, max_depth: int = 50,
           seed: int = 0, row_offset: int = 0, row_stride: int = 1, want_rgb: bool = True,
           cull: bool = True, fixpoint: bool = True, cull_stats: bool = False, out=None):
    """One-shot render of the owned rows on the default device (RT_DEVICE).

    cull=False forces the linear sweep; fixpoint=False traces provably trapped
    paths to max_depth. Neither changes a bit of the output.
    cull_stats=True counts the executed sphere / box tests (tests_executed,
    box_tests; 0 otherwise) with the slower counting kernel, same bits.
    out=(accum, rgb8 or None): write into these arrays (e.g. host_array(...),
    which the device writes directly) instead of new ones; out=(None, rgb8):
    the write_color bytes only, what the reference's main() prints (the FP64
    sums then stay on the device: 2.9 MB crosses the link for C3, not 26 MB).

    Returns (accum[rows, W, 3] float64 or None, rgb8[rows, W, 3] uint8 or None, stats dict).
    """
    L = _lib.load()
    sp, n = _spheres(spheres)
    cam = _camera(camera)
    p = params(width, height, spp, max_depth, seed, row_offset, row_stride,
               (0 if cull else FLAG_NO_CULL) | (0 if fixpoint else FLAG_NO_FIXPOINT)
               | (FLAG_CULL_STATS if cull_stats else 0))
    # a shard that owns no rows (row_offset >= height: more ranks than rows)
    # renders nothing and returns empty [0, W, 3] blocks
    rows = max(0, L.rt_rows_owned(height, row_offset, row_stride))
    acc, rgb = _out_arrays(out, rows, width, want_rgb)
    st = RtStats()
    check(L.rt_render(sp, n, C.byref(cam), C.byref(p),
                      acc.ctypes.data_as(C.POINTER(C.c_double)) if acc is not None else None,
                      rgb.ctypes.data_as(C.POINTER(C.c_ubyte)) if rgb is not None else None,
                      C.byref(st)), "rt_render")
    return acc, rgb, stats_dict(st)


def render_materials(spheres, materials, camera: LensCamera, width: int, height: int, spp: int,
                     max_depth: int = 50, seed: int = 0, row_offset: int = 0, row_stride: int = 1,
                     want_rgb: bool = True, cull: bool = True):
    """One-shot render with the material integrator (rt_render_materials).
    Returns (accum[rows, W, 3] float64, rgb8 or None, stats dict)."""
    L = _lib.load()
    sp, n = _spheres(spheres)
    mt, nm = _materials(materials)
    if nm != n:
        raise ValueError("one material per sphere")
    cam = camera.to_c()
    p = params(width, height, spp, max_depth, seed, row_offset, row_stride,
               FLAG_MATERIALS | (0 if cull else FLAG_NO_CULL))
    rows = max(0, L.rt_rows_owned(height, row_offset, row_stride))
    acc = np.zeros((rows, width, 3), dtype=np.float64)
    rgb = np.zeros((rows, width, 3), dtype=np.uint8) if want_rgb else None
    st = RtStats()
    check(L.rt_render_materials(sp, mt, n, C.byref(cam), C.byref(p),
                                acc.ctypes.data_as(C.POINTER(C.c_double)),
                                rgb.ctypes.data_as(C.POINTER(C.c_ubyte)) if rgb is not None
                                else None, C.byref(st)), "rt_render_materials")
    return acc, rgb, stats_dict(st)


def set_tuning(name: str, value: float, ctx: Optional["Context"] = None) -> None:
    """rt_context_set_tuning: a measurement / test knob (include/rt.h) of one
    context, or (ctx=None) the process defaults that new contexts and the
    one-shot entries take. Every knob keeps the output bit-identical."""
    L = _lib.load()
    check(L.rt_context_set_tuning(ctx.handle if ctx is not None else None, name.encode(),
                                  float(value)), "rt_context_set_tuning")


def get_tuning(name: str, ctx: Optional["Context"] = None) -> float:
    v = C.c_double()
    check(_lib.load().rt_context_get_tuning(ctx.handle if ctx is not None else None,
                                            name.encode(), C.byref(v)), "rt_context_get_tuning")
    return v.value


@contextmanager
def tuning(**knobs):
    """Set process-default knobs for the duration of a block (tests, A/B
    scripts), then restore the previous values."""
    old = {k: get_tuning(k) for k in knobs}
    try:
        for k, v in knobs.items():
            set_tuning(k, v)
        yield
    finally:
        for k, v in old.items():
            set_tuning(k, v)


def quantize(accum: np.ndarray, spp: int) -> np.ndarray:
    """write_color (color.h:8-24) on host accumulators."""
    acc = np.ascontiguousarray(accum, dtype=np.float64)
    out = np.zeros(acc.shape, dtype=np.uint8)
    rows, w = acc.shape[0], acc.shape[1]
    check(_lib.load().rt_quantize_ppm(acc.ctypes.data_as(C.POINTER(C.c_double)), w, rows, spp,
                                      out.ctypes.data_as(C.POINTER(C.c_ubyte))),
          "rt_quantize_ppm")
    return out


class Context:
    """An rt_context on one HIP device: device-resident scene and buffers."""

    def __init__(self, device: int = 0):
        self._L = _lib.load()
        h = C.c_void_p()
        check(self._L.rt_context_create(device, C.byref(h)), "rt_context_create")
        self.handle = h
        self.device = device

    def set_scene(self, spheres, camera) -> None:
        sp, n = _spheres(spheres)
        cam = _camera(camera)
        check(self._L.rt_context_set_scene(self.handle, sp, n, C.byref(cam)),
              "rt_context_set_scene")

    def set_materials(self, materials, camera: Optional[LensCamera]) -> None:
        """Materials (n, 6) for the scene's spheres and the lens camera of
        renders with FLAG_MATERIALS; materials=None clears them."""
        if materials is None:
            check(self._L.rt_context_set_materials(self.handle, None, 0, None),
                  "rt_context_set_materials")
            return
        mt, n = _materials(materials)
        cam = camera.to_c()
        check(self._L.rt_context_set_materials(self.handle, mt, n, C.byref(cam)),
              "rt_context_set_materials")

    def render_device(self, p: RtParams, d_accum: int = 0, d_rgb8: int = 0,
                      stream: int = 0) -> None:
        """Enqueue a render into device pointers (ints, e.g. tensor.data_ptr())."""
        check(self._L.rt_render_device(self.handle, C.byref(p), d_accum or None,
                                       d_rgb8 or None, stream or None), "rt_render_device")

    def render_device_frames(self, p: RtParams, nframes: int, d_accum=None, d_rgb8=None,
                             stream: int = 0) -> None:
        """Enqueue nframes renders in one trace launch per sample chunk: frame f
        is the frame of seed p.seed + f; d_accum / d_rgb8: sequences of nframes
        device pointers (ints, 0 = none) or None."""
        def arr(ptrs):
            if ptrs is None:
                return None
            if len(ptrs) != nframes:
                raise ValueError("one pointer per frame")
            return (C.c_void_p * nframes)(*[x or None for x in ptrs])
        check(self._L.rt_render_device_frames(self.handle, C.byref(p), nframes, arr(d_accum),
                                              arr(d_rgb8), stream or None),
              "rt_render_device_frames")

    def debug_fail_after_trace(self, chunk: int) -> None:
        """Fault injection (tests only): the next render fails after sample
        chunk `chunk`'s trace launch, before its reduce (rt_debug_fail_after_trace)."""
        check(self._L.rt_debug_fail_after_trace(self.handle, chunk), "rt_debug_fail_after_trace")

    def set_row_pitch(self, accum_pitch: int = 0, rgb8_pitch: int = 0) -> None:
        """rt_context_set_row_pitch: the shard's output rows this many doubles /
        bytes apart (0 = packed), so shards can write one frame in place."""
        check(self._L.rt_context_set_row_pitch(self.handle, accum_pitch, rgb8_pitch),
              "rt_context_set_row_pitch")

    def wait_drain(self, stream: int) -> None:
        """rt_context_wait_drain: `stream` waits until this context's last
        enqueued trace launch has emptied its work queue, so a render enqueued
        on it next (another context's frame) starts in this launch's tail."""
        check(self._L.rt_context_wait_drain(self.handle, stream or None), "rt_context_wait_drain")

    def set_tuning(self, name: str, value: float) -> None:
        """rt_context_set_tuning on this context (measurement / test knobs)."""
        set_tuning(name, value, self)

    def get_tuning(self, name: str) -> float:
        return get_tuning(name, self)

    def stream(self) -> int:
        """The context's own hipStream_t (as an int), used for stream=0."""
        return self._L.rt_context_stream(self.handle) or 0

    def sync_stats(self) -> dict:
        st = RtStats()
        check(self._L.rt_context_sync_stats(self.handle, C.byref(st)), "rt_context_sync_stats")
        return stats_dict(st)

    def quantize_device(self, d_accum: int, width: int, rows: int, spp: int, d_rgb8: int,
                        stream: int = 0) -> None:
        check(self._L.rt_quantize_device(self.handle, d_accum, width, rows, spp, d_rgb8,
                                         stream or None), "rt_quantize_device")

    def close(self) -> None:
        if self.handle:
            self._L.rt_context_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class DeviceGroup:
    """rt_group (include/rt.h): one frame over several devices natively, one
    context and host thread per member, interleaved rows gathered into
    reference pixel order in host memory. Members may repeat a device."""

    def __init__(self, devices):
        self._L = _lib.load()
        devs = (C.c_int * len(devices))(*devices)
        h = C.c_void_p()
        check(self._L.rt_group_create(devs, len(devices), C.byref(h)), "rt_group_create")
        self.handle = h
        self.devices = list(devices)

    def set_scene(self, spheres, camera) -> None:
        sp, n = _spheres(spheres)
        cam = _camera(camera)
        check(self._L.rt_group_set_scene(self.handle, sp, n, C.byref(cam)), "rt_group_set_scene")

    def render(self, width: int, height: int, spp: int, max_depth: int = 50, seed: int = 0,
               row_offset: int = 0, row_stride: int = 1, flags: int = 0, want_rgb: bool = True,
               out=None):
        """Returns (accum[rows, W, 3], rgb8 or None, stats) of the shard
        (out=(accum, rgb8 or None): into these arrays, as render())."""
        p = params(width, height, spp, max_depth, seed, row_offset, row_stride, flags)
        rows = max(0, self._L.rt_rows_owned(height, row_offset, row_stride))
        acc, rgb = _out_arrays(out, rows, width, want_rgb)
        if acc is None:
            raise ValueError("rt_group_render needs the accum array")
        st = RtStats()
        check(self._L.rt_group_render(self.handle, C.byref(p),
                                      acc.ctypes.data_as(C.POINTER(C.c_double)),
                                      rgb.ctypes.data_as(C.POINTER(C.c_ubyte))
                                      if rgb is not None else None, C.byref(st)),
              "rt_group_render")
        return acc, rgb, stats_dict(st)

    def close(self) -> None:
        if self.handle:
            self._L.rt_group_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def render_devices(spheres, camera, width: int, height: int, spp: int, devices,
                   max_depth: int = 50, seed: int = 0, row_offset: int = 0, row_stride: int = 1):
    """rt_render_devices: one-shot render of the shard over `devices`."""
    L = _lib.load()
    sp, n = _spheres(spheres)
    cam = _camera(camera)
    p = params(width, height, spp, max_depth, seed, row_offset, row_stride)
    rows = max(0, L.rt_rows_owned(height, row_offset, row_stride))
    acc = np.zeros((rows, width, 3), dtype=np.float64)
    rgb = np.zeros((rows, width, 3), dtype=np.uint8)
    st = RtStats()
    devs = (C.c_int * len(devices))(*devices)
    check(L.rt_render_devices(sp, n, C.byref(cam), C.byref(p), devs, len(devices),
                              acc.ctypes.data_as(C.POINTER(C.c_double)),
                              rgb.ctypes.data_as(C.POINTER(C.c_ubyte)), C.byref(st)),
          "rt_render_devices")
    return acc, rgb, stats_dict(st)


def ppm_p3(rgb8: np.ndarray) -> bytes:
    """P3 text exactly as main.cc:70 and color.h:21-23 write it."""
    rows, w = rgb8.shape[0], rgb8.shape[1]
    flat = np.asarray(rgb8, dtype=np.uint8).reshape(-1, 3)
    body = "".join(f"{r} {g} {b}\n" for r, g, b in flat.tolist())
    return f"P3\n{w} {rows}\n255\n{body}".encode()


def write_ppm(path: str, rgb8: np.ndarray, binary: bool = False) -> None:
    """Write P3 (reference format) or P6 (binary) PPM."""
    rows, w = rgb8.shape[0], rgb8.shape[1]
    with open(path, "wb") as f:
        if binary:
            f.write(f"P6\n{w} {rows}\n255\n".encode())
            f.write(np.ascontiguousarray(rgb8, dtype=np.uint8).tobytes())
        else:
            f.write(ppm_p3(rgb8))


def device_count() -> int:
    return _lib.load().rt_device_count()


def probe_f64(op: int, x: np.ndarray, y: Optional[np.ndarray] = None) -> np.ndarray:
    """Run one binary64 primitive on the device (numerics tests)."""
    x = np.ascontiguousarray(x, dtype=np.float64)
    y = np.ascontiguousarray(np.zeros_like(x) if y is None else y, dtype=np.float64)
    out = np.zeros_like(x)
    P = C.POINTER(C.c_double)
    check(_lib.load().rt_debug_probe_f64(op, x.ctypes.data_as(P), y.ctypes.data_as(P),
                                         out.ctypes.data_as(P), len(x)), "rt_debug_probe_f64")
    return out


def world_hit(spheres, rays: np.ndarray, cull: bool = True,
              hints: Optional[np.ndarray] = None) -> np.ndarray:
    """hittable_list::hit on the device for rays[k] = (o, d, tmin, tmax);
    returns out[k] = (index, p, normal, t, front_face) (debug / KAT entry).
    With cull, rays with tmin == 0, tmax == inf go through the BVH path;
    hints[k] (optional, -1 = none) is the sphere ray k starts on, tested first
    as the trace kernel tests a bounce ray's previous hit."""
    sp, n = _spheres(spheres)
    r = np.ascontiguousarray(rays, dtype=np.float64).reshape(-1, 8)
    out = np.zeros((len(r), 9), dtype=np.float64)
    P = C.POINTER(C.c_double)
    if hints is None:
        check(_lib.load().rt_debug_world_hit(sp, n, r.ctypes.data_as(P), len(r),
                                             out.ctypes.data_as(P), 1 if cull else 0),
              "rt_debug_world_hit")
        return out
    h = np.ascontiguousarray(hints, dtype=np.int32).reshape(-1)
    if len(h) != len(r):
        raise ValueError("hints: one per ray")
    check(_lib.load().rt_debug_world_hit_hint(sp, n, r.ctypes.data_as(P),
                                              h.ctypes.data_as(C.POINTER(C.c_int)), len(r),
                                              out.ctypes.data_as(P), 1 if cull else 0),
          "rt_debug_world_hit_hint")
    return out
