"""ORACLE — test infrastructure only.

ctypes binding to ``oracle/build/liboracle.so`` (the plain-C restatement of the
reference hot path, ``oracle/rt_oracle.c``) and a runner for
``oracle/_ref/ref_render`` (the reference's own sources behind a driver).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg import this package, and only as the checker: the product
(``petershirleyraytracer_amd``) never imports, links or executes anything here.
"""
from __future__ import annotations

import ctypes as C
import json
import os
import subprocess
from typing import Optional, Sequence

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "liboracle.so")
REF_BIN = os.path.join(HERE, "_ref", "ref_render")

RNG_COUNTER = 0
RNG_GLIBC = 1


class Sphere(C.Structure):
    _fields_ = [("cx", C.c_double), ("cy", C.c_double), ("cz", C.c_double), ("r", C.c_double)]


class Camera(C.Structure):
    _fields_ = [
        ("origin", C.c_double * 3),
        ("lower_left", C.c_double * 3),
        ("horizontal", C.c_double * 3),
        ("vertical", C.c_double * 3),
    ]


class Params(C.Structure):
    _fields_ = [
        ("width", C.c_int),
        ("height", C.c_int),
        ("spp", C.c_int),
        ("max_depth", C.c_int),
        ("seed", C.c_uint64),
        ("row_offset", C.c_int),
        ("row_stride", C.c_int),
        ("flags", C.c_uint),
    ]


class Material(C.Structure):
    _fields_ = [("kind", C.c_int), ("reserved", C.c_int), ("albedo", C.c_double * 3),
                ("fuzz", C.c_double), ("ir", C.c_double)]


class CameraLens(C.Structure):
    _fields_ = [("base", Camera), ("u", C.c_double * 3), ("v", C.c_double * 3),
                ("lens_radius", C.c_double)]


class Bounce(C.Structure):
    _fields_ = [
        ("o", C.c_double * 3),
        ("d", C.c_double * 3),
        ("t", C.c_double),
        ("index", C.c_int32),
        ("front_face", C.c_int32),
        ("draws_after", C.c_uint64),
    ]


_lib = None


def build() -> None:
    """Compile liboracle.so (and _ref/ref_render when /root/reference exists)."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        L.oracle_render.argtypes = [
            C.POINTER(Sphere), C.c_int, C.POINTER(Camera), C.POINTER(Params), C.c_int, C.c_int,
            C.POINTER(C.c_double), C.POINTER(C.c_ubyte), C.POINTER(C.c_uint64)]
        L.oracle_render_pixels.argtypes = [
            C.POINTER(Sphere), C.c_int, C.POINTER(Camera), C.POINTER(Params),
            C.POINTER(C.c_int), C.POINTER(C.c_int), C.c_int, C.POINTER(C.c_double),
            C.POINTER(C.c_uint64)]
        L.oracle_trace_sample.argtypes = [
            C.POINTER(Sphere), C.c_int, C.POINTER(Camera), C.POINTER(Params), C.c_int, C.c_int,
            C.c_int, C.POINTER(C.c_double), C.POINTER(Bounce), C.c_int]
        L.oracle_sphere_hit.argtypes = [C.POINTER(Sphere), C.POINTER(C.c_double),
                                        C.POINTER(C.c_double), C.c_double, C.c_double,
                                        C.POINTER(C.c_double)]
        L.oracle_world_hit.argtypes = [C.POINTER(Sphere), C.c_int, C.POINTER(C.c_double),
                                       C.POINTER(C.c_double), C.c_double, C.c_double,
                                       C.POINTER(C.c_double)]
        L.oracle_counter_draws.argtypes = [C.c_uint64, C.c_uint32, C.c_uint32, C.c_int,
                                           C.POINTER(C.c_int32)]
        L.oracle_counter_draws.restype = None
        L.oracle_glibc_draws.argtypes = [C.c_uint, C.c_int, C.POINTER(C.c_int32)]
        L.oracle_glibc_draws.restype = None
        L.oracle_camera_default.argtypes = [C.POINTER(Camera)]
        L.oracle_camera_default.restype = None
        L.oracle_camera_look_at.argtypes = [C.POINTER(C.c_double)] * 3 + [
            C.c_double, C.c_double, C.POINTER(Camera)]
        L.oracle_camera_look_at.restype = None
        L.oracle_scene_random_spheres.argtypes = [C.c_uint, C.POINTER(Sphere), C.c_int]
        L.oracle_quantize.argtypes = [C.POINTER(C.c_double), C.c_int, C.c_int, C.c_int,
                                      C.POINTER(C.c_ubyte)]
        L.oracle_rows_owned.argtypes = [C.c_int, C.c_int, C.c_int]
        # rt_oracle_mat.c (materials extension, parity unpinned)
        L.oracle_render_mat.argtypes = [
            C.POINTER(Sphere), C.POINTER(Material), C.c_int, C.POINTER(CameraLens),
            C.POINTER(Params), C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_uint64)]
        L.oracle_scene_book_final.argtypes = [C.c_uint, C.POINTER(Sphere), C.POINTER(Material),
                                              C.c_int]
        L.oracle_camera_look_at_lens.argtypes = [C.POINTER(C.c_double)] * 3 + [
            C.c_double] * 4 + [C.POINTER(CameraLens)]
        L.oracle_camera_look_at_lens.restype = None
        _lib = L
    return _lib


# ---- helpers -----------------------------------------------------------------

def spheres_array(spheres) -> "C.Array":
    """spheres: (n,4) array-like of (cx, cy, cz, r)."""
    arr = np.ascontiguousarray(np.asarray(spheres, dtype=np.float64).reshape(-1, 4))
    out = (Sphere * max(1, len(arr)))()
    C.memmove(out, arr.ctypes.data, arr.nbytes)
    return out, len(arr)


def camera_to_array(cam: Camera) -> np.ndarray:
    return np.array([list(cam.origin), list(cam.lower_left), list(cam.horizontal),
                     list(cam.vertical)], dtype=np.float64)


def camera_from_array(a) -> Camera:
    a = np.asarray(a, dtype=np.float64).reshape(4, 3)
    c = Camera()
    for k in range(3):
        c.origin[k], c.lower_left[k], c.horizontal[k], c.vertical[k] = a[0, k], a[1, k], a[2, k], a[3, k]
    return c


def make_params(width, height, spp, max_depth=50, seed=0, row_offset=0, row_stride=1) -> Params:
    return Params(width, height, spp, max_depth, seed, row_offset, row_stride, 0)


def rows_owned(height, row_offset=0, row_stride=1) -> int:
    return lib().oracle_rows_owned(height, row_offset, row_stride)


def camera_default() -> np.ndarray:
    c = Camera()
    lib().oracle_camera_default(C.byref(c))
    return camera_to_array(c)


def camera_look_at(lookfrom=(13, 2, 3), lookat=(0, 0, 0), vup=(0, 1, 0), vfov=20.0,
                   aspect=1.5) -> np.ndarray:
    c = Camera()
    f = (C.c_double * 3)(*lookfrom)
    a = (C.c_double * 3)(*lookat)
    u = (C.c_double * 3)(*vup)
    lib().oracle_camera_look_at(f, a, u, vfov, aspect, C.byref(c))
    return camera_to_array(c)


def scene_two_spheres() -> np.ndarray:
    """main.cc:61-63"""
    return np.array([[0.0, 0.0, -1.0, 0.5], [0.0, -100.5, 0.0, 100.0]])


def scene_random_spheres(seed: int = 1) -> np.ndarray:
    buf = (Sphere * 1024)()
    n = lib().oracle_scene_random_spheres(seed, buf, 1024)
    return np.frombuffer(buf, dtype=np.float64, count=n * 4).reshape(n, 4).copy()


def render(spheres, camera, width, height, spp, max_depth=50, seed=0, row_offset=0,
           row_stride=1, rng=RNG_COUNTER, threads=1):
    """Returns (accum[rows, W, 3] float64, rgb8[rows, W, 3] uint8, rays)."""
    sp, n = spheres_array(spheres)
    cam = camera_from_array(camera)
    p = make_params(width, height, spp, max_depth, seed, row_offset, row_stride)
    rows = rows_owned(height, row_offset, row_stride)
    acc = np.zeros((rows, width, 3), dtype=np.float64)
    rgb = np.zeros((rows, width, 3), dtype=np.uint8)
    rays = C.c_uint64(0)
    rc = lib().oracle_render(sp, n, C.byref(cam), C.byref(p), rng, threads,
                             acc.ctypes.data_as(C.POINTER(C.c_double)),
                             rgb.ctypes.data_as(C.POINTER(C.c_ubyte)), C.byref(rays))
    if rc != 0:
        raise RuntimeError(f"oracle_render failed: {rc}")
    return acc, rgb, rays.value


def render_pixels(spheres, camera, width, height, spp, ii: Sequence[int], jj: Sequence[int],
                  max_depth=50, seed=0):
    """Counter-mode pixel_color for reference pixel coordinates (i, j)."""
    sp, n = spheres_array(spheres)
    cam = camera_from_array(camera)
    p = make_params(width, height, spp, max_depth, seed)
    ii = np.ascontiguousarray(ii, dtype=np.int32)
    jj = np.ascontiguousarray(jj, dtype=np.int32)
    out = np.zeros((len(ii), 3), dtype=np.float64)
    rays = C.c_uint64(0)
    rc = lib().oracle_render_pixels(sp, n, C.byref(cam), C.byref(p),
                                    ii.ctypes.data_as(C.POINTER(C.c_int)),
                                    jj.ctypes.data_as(C.POINTER(C.c_int)), len(ii),
                                    out.ctypes.data_as(C.POINTER(C.c_double)), C.byref(rays))
    if rc != 0:
        raise RuntimeError(f"oracle_render_pixels failed: {rc}")
    return out, rays.value


def trace_sample(spheres, camera, width, height, i, j, s, max_depth=50, seed=0, cap=64):
    sp, n = spheres_array(spheres)
    cam = camera_from_array(camera)
    p = make_params(width, height, 1, max_depth, seed)
    col = (C.c_double * 3)()
    tr = (Bounce * cap)()
    ln = lib().oracle_trace_sample(sp, n, C.byref(cam), C.byref(p), i, j, s, col, tr, cap)
    bounces = [dict(o=list(b.o), d=list(b.d), t=b.t, index=b.index, front_face=b.front_face,
                    draws_after=b.draws_after) for b in tr[:min(ln, cap)]]
    return list(col), bounces


def sphere_hit(sphere, o, d, tmin, tmax):
    s = Sphere(*sphere)
    out = (C.c_double * 8)()
    hit = lib().oracle_sphere_hit(C.byref(s), (C.c_double * 3)(*o), (C.c_double * 3)(*d),
                                  tmin, tmax, out)
    return bool(hit), list(out)


def world_hit(spheres, o, d, tmin, tmax):
    sp, n = spheres_array(spheres)
    out = (C.c_double * 8)()
    idx = lib().oracle_world_hit(sp, n, (C.c_double * 3)(*o), (C.c_double * 3)(*d), tmin, tmax, out)
    return idx, list(out)


def counter_draws(seed, pixel, sample, count) -> np.ndarray:
    out = np.zeros(count, dtype=np.int32)
    lib().oracle_counter_draws(seed, pixel, sample, count, out.ctypes.data_as(C.POINTER(C.c_int32)))
    return out


def glibc_draws(seed, count) -> np.ndarray:
    out = np.zeros(count, dtype=np.int32)
    lib().oracle_glibc_draws(seed, count, out.ctypes.data_as(C.POINTER(C.c_int32)))
    return out


def quantize(accum: np.ndarray, spp: int) -> np.ndarray:
    acc = np.ascontiguousarray(accum, dtype=np.float64)
    rows, w = acc.shape[0], acc.shape[1]
    out = np.zeros(acc.shape, dtype=np.uint8)
    lib().oracle_quantize(acc.ctypes.data_as(C.POINTER(C.c_double)), w, rows, spp,
                          out.ctypes.data_as(C.POINTER(C.c_ubyte)))
    return out


def ppm_p3(rgb8: np.ndarray) -> bytes:
    """P3 text exactly as main.cc:70 + color.h:21-23 print it."""
    rows, w = rgb8.shape[0], rgb8.shape[1]
    lines = [f"P3\n{w} {rows}\n255\n"]
    flat = rgb8.reshape(-1, 3)
    lines.extend(f"{r} {g} {b}\n" for r, g, b in flat.tolist())
    return "".join(lines).encode()


# ---- the reference itself ----------------------------------------------------

def have_ref() -> bool:
    return os.path.exists(REF_BIN)


def run_ref(args: Sequence[str], timeout: Optional[float] = None):
    """Run oracle/_ref/ref_render; returns (stdout bytes, stats dict)."""
    r = subprocess.run([REF_BIN, *args], capture_output=True, timeout=timeout, check=True)
    stats = {}
    for line in r.stderr.decode().splitlines():
        line = line.strip()
        if line.startswith("{"):
            stats = json.loads(line)
    return r.stdout, stats


# ---- materials extension (rt_oracle_mat.c; DESIGN.md §14, parity unpinned) ----

def materials_struct(mats):
    """mats: (n, 6) rows (kind, albedo r, g, b, fuzz, ir)."""
    a = np.asarray(mats, dtype=np.float64).reshape(-1, 6)
    out = (Material * max(1, len(a)))()
    for k, row in enumerate(a):
        out[k].kind = int(row[0])
        out[k].albedo[0], out[k].albedo[1], out[k].albedo[2] = row[1], row[2], row[3]
        out[k].fuzz, out[k].ir = row[4], row[5]
    return out, len(a)


def lens_to_dict(c: CameraLens) -> dict:
    return dict(base=camera_to_array(c.base), u=np.array(list(c.u)), v=np.array(list(c.v)),
                lens_radius=c.lens_radius)


def lens_from(base, u, v, lens_radius) -> CameraLens:
    c = CameraLens()
    c.base = camera_from_array(base)
    for k in range(3):
        c.u[k], c.v[k] = float(u[k]), float(v[k])
    c.lens_radius = float(lens_radius)
    return c


def camera_look_at_lens(lookfrom=(13, 2, 3), lookat=(0, 0, 0), vup=(0, 1, 0), vfov=20.0,
                        aspect=1.5, aperture=0.1, focus_dist=10.0) -> dict:
    c = CameraLens()
    d3 = C.c_double * 3
    lib().oracle_camera_look_at_lens(d3(*lookfrom), d3(*lookat), d3(*vup), vfov, aspect,
                                     aperture, focus_dist, C.byref(c))
    return lens_to_dict(c)


def scene_book_final(seed: int = 1):
    sp = (Sphere * 1024)()
    mt = (Material * 1024)()
    n = lib().oracle_scene_book_final(seed, sp, mt, 1024)
    spheres = np.frombuffer(sp, dtype=np.float64, count=n * 4).reshape(n, 4).copy()
    mats = np.array([[mt[k].kind, *list(mt[k].albedo), mt[k].fuzz, mt[k].ir] for k in range(n)],
                    dtype=np.float64).reshape(n, 6)
    return spheres, mats


def render_mat(spheres, mats, lens: dict, width, height, spp, max_depth=50, seed=0,
               row_offset=0, row_stride=1, threads=1):
    """The book's material integrator over the counter stream.
    Returns (accum[rows, W, 3] float64, rays)."""
    sp, n = spheres_array(spheres)
    mt, nm = materials_struct(mats)
    assert nm == n
    cam = lens_from(lens["base"], lens["u"], lens["v"], lens["lens_radius"])
    p = make_params(width, height, spp, max_depth, seed, row_offset, row_stride)
    rows = rows_owned(height, row_offset, row_stride)
    acc = np.zeros((rows, width, 3), dtype=np.float64)
    rays = C.c_uint64(0)
    rc = lib().oracle_render_mat(sp, mt, n, C.byref(cam), C.byref(p), threads,
                                 acc.ctypes.data_as(C.POINTER(C.c_double)), C.byref(rays))
    if rc != 0:
        raise RuntimeError(f"oracle_render_mat failed: {rc}")
    return acc, rays.value
