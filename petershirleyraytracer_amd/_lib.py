"""ctypes binding of libpsrt.so (include/rt.h).

The product path is the HIP library: if ``lib/libpsrt.so`` is missing or has
no HIP device, calls raise — there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os

from .build import LIB

RT_OK = 0
# include/rt.h RT_ABI_VERSION: the struct layouts below (RtStats grew in ABI 5)
# and the entry points (rt_host_alloc / rt_host_free arrived in ABI 6,
# rt_context_wait_drain in ABI 7)
# are that version's, so a library of another version is refused at load
# (tests/test_abi.py checks this constant against the header)
ABI_VERSION = 7
ERRORS = {-1: "RT_E_INVALID", -2: "RT_E_HIP", -3: "RT_E_NODEVICE", -4: "RT_E_NOMEM",
          -5: "RT_E_SCENE"}

# Every symbol include/rt.h declares (checked by tests/test_abi.py).
EXPORTS = [
    "rt_rows_owned", "rt_render", "rt_quantize_ppm", "rt_context_create", "rt_context_destroy",
    "rt_context_set_scene", "rt_render_device", "rt_render_device_frames", "rt_context_stream", "rt_context_sync_stats", "rt_quantize_device",
    "rt_camera_default", "rt_camera_look_at", "rt_scene_two_spheres", "rt_scene_random_spheres",
    "rt_scene_parse", "rt_scene_load", "rt_scene_format",
    "rt_last_error", "rt_abi_version", "rt_device_count", "rt_build_info", "rt_debug_probe_f64",
    "rt_debug_world_hit", "rt_debug_world_hit_hint", "rt_debug_fail_after_trace",
    "rt_camera_look_at_lens", "rt_scene_book_final", "rt_context_set_materials",
    "rt_render_materials", "rt_context_set_tuning", "rt_context_get_tuning",
    "rt_group_create", "rt_group_destroy", "rt_group_size", "rt_group_context",
    "rt_group_set_scene", "rt_group_render", "rt_render_devices", "rt_host_alloc", "rt_host_free",
    "rt_host_register", "rt_host_unregister", "rt_context_set_row_pitch",
    "rt_context_wait_drain",
]


class RtSphere(C.Structure):
    _fields_ = [("cx", C.c_double), ("cy", C.c_double), ("cz", C.c_double), ("r", C.c_double)]


class RtCamera(C.Structure):
    _fields_ = [("origin", C.c_double * 3), ("lower_left", C.c_double * 3),
                ("horizontal", C.c_double * 3), ("vertical", C.c_double * 3)]


class RtParams(C.Structure):
    _fields_ = [("width", C.c_int), ("height", C.c_int), ("spp", C.c_int),
                ("max_depth", C.c_int), ("seed", C.c_uint64), ("row_offset", C.c_int),
                ("row_stride", C.c_int), ("flags", C.c_uint)]


class RtMaterial(C.Structure):
    _fields_ = [("kind", C.c_int), ("reserved", C.c_int), ("albedo", C.c_double * 3),
                ("fuzz", C.c_double), ("ir", C.c_double)]


class RtCameraLens(C.Structure):
    _fields_ = [("base", RtCamera), ("u", C.c_double * 3), ("v", C.c_double * 3),
                ("lens_radius", C.c_double)]


class RtStats(C.Structure):
    _fields_ = [("samples", C.c_uint64), ("rays", C.c_uint64), ("sphere_tests", C.c_uint64),
                ("tests_executed", C.c_uint64), ("box_tests", C.c_uint64),
                ("kernel_ms", C.c_double), ("total_ms", C.c_double), ("rays_traced", C.c_uint64),
                ("prerejects", C.c_uint64), ("root_box_tests", C.c_uint64)]


class RtError(RuntimeError):
    pass


_lib = None


def load(build_if_missing: bool = False):
    """Load libpsrt.so. Raises if it is absent (unless asked to build it)."""
    global _lib
    if _lib is not None:
        return _lib
    # One HIP runtime per process: torch ships its own libamdhip64 (SONAME
    # libamdhip64.so.7, NEEDed by torch as "libamdhip64.so"). Loaded first, it
    # also satisfies libpsrt.so's NEEDED libamdhip64.so.7; loaded after ours,
    # torch would map a second runtime that cannot see the GPU.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib_path = os.environ.get("PSRT_LIB", LIB)  # A/B builds (tuning only)
    if not os.path.exists(lib_path):
        if build_if_missing:
            from .build import build_lib
            build_lib()
        else:
            raise RtError(f"libpsrt.so not built ({LIB}); run __graft_entry__.build() or "
                          f"python -m petershirleyraytracer_amd.build")
    L = C.CDLL(lib_path)
    P = C.POINTER
    sig = {
        "rt_rows_owned": ([C.c_int, C.c_int, C.c_int], C.c_int),
        "rt_render": ([P(RtSphere), C.c_int, P(RtCamera), P(RtParams), P(C.c_double),
                       P(C.c_ubyte), P(RtStats)], C.c_int),
        "rt_quantize_ppm": ([P(C.c_double), C.c_int, C.c_int, C.c_int, P(C.c_ubyte)], C.c_int),
        "rt_context_create": ([C.c_int, P(C.c_void_p)], C.c_int),
        "rt_context_destroy": ([C.c_void_p], C.c_int),
        "rt_context_set_scene": ([C.c_void_p, P(RtSphere), C.c_int, P(RtCamera)], C.c_int),
        "rt_render_device": ([C.c_void_p, P(RtParams), C.c_void_p, C.c_void_p, C.c_void_p],
                             C.c_int),
        "rt_render_device_frames": ([C.c_void_p, P(RtParams), C.c_int, P(C.c_void_p),
                                     P(C.c_void_p), C.c_void_p], C.c_int),
        "rt_context_sync_stats": ([C.c_void_p, P(RtStats)], C.c_int),
        "rt_context_stream": ([C.c_void_p], C.c_void_p),
        "rt_quantize_device": ([C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p,
                                C.c_void_p], C.c_int),
        "rt_camera_default": ([P(RtCamera)], C.c_int),
        "rt_camera_look_at": ([P(C.c_double), P(C.c_double), P(C.c_double), C.c_double,
                               C.c_double, P(RtCamera)], C.c_int),
        "rt_scene_two_spheres": ([P(RtSphere), C.c_int], C.c_int),
        "rt_scene_random_spheres": ([C.c_uint, P(RtSphere), C.c_int], C.c_int),
        "rt_scene_parse": ([C.c_char_p, P(RtSphere), C.c_int, P(RtCamera), P(RtParams)],
                           C.c_int),
        "rt_scene_load": ([C.c_char_p, P(RtSphere), C.c_int, P(RtCamera), P(RtParams)],
                          C.c_int),
        "rt_scene_format": ([P(RtSphere), C.c_int, P(RtCamera), P(RtParams), C.c_char_p,
                             C.c_size_t], C.c_longlong),
        "rt_last_error": ([], C.c_char_p),
        "rt_abi_version": ([], C.c_int),
        "rt_device_count": ([], C.c_int),
        "rt_build_info": ([], C.c_char_p),
        "rt_debug_probe_f64": ([C.c_int, P(C.c_double), P(C.c_double), P(C.c_double), C.c_int],
                               C.c_int),
        "rt_debug_world_hit": ([P(RtSphere), C.c_int, P(C.c_double), C.c_int, P(C.c_double),
                                C.c_int], C.c_int),
        "rt_debug_world_hit_hint": ([P(RtSphere), C.c_int, P(C.c_double), P(C.c_int), C.c_int,
                                     P(C.c_double), C.c_int], C.c_int),
        "rt_debug_fail_after_trace": ([C.c_void_p, C.c_int], C.c_int),
        "rt_camera_look_at_lens": ([P(C.c_double), P(C.c_double), P(C.c_double), C.c_double,
                                    C.c_double, C.c_double, C.c_double, P(RtCameraLens)],
                                   C.c_int),
        "rt_scene_book_final": ([C.c_uint, P(RtSphere), P(RtMaterial), C.c_int], C.c_int),
        "rt_context_set_materials": ([C.c_void_p, P(RtMaterial), C.c_int, P(RtCameraLens)],
                                     C.c_int),
        "rt_render_materials": ([P(RtSphere), P(RtMaterial), C.c_int, P(RtCameraLens),
                                 P(RtParams), P(C.c_double), P(C.c_ubyte), P(RtStats)], C.c_int),
        "rt_context_set_tuning": ([C.c_void_p, C.c_char_p, C.c_double], C.c_int),
        "rt_context_get_tuning": ([C.c_void_p, C.c_char_p, P(C.c_double)], C.c_int),
        "rt_group_create": ([P(C.c_int), C.c_int, P(C.c_void_p)], C.c_int),
        "rt_group_destroy": ([C.c_void_p], C.c_int),
        "rt_group_size": ([C.c_void_p], C.c_int),
        "rt_group_context": ([C.c_void_p, C.c_int], C.c_void_p),
        "rt_group_set_scene": ([C.c_void_p, P(RtSphere), C.c_int, P(RtCamera)], C.c_int),
        "rt_group_render": ([C.c_void_p, P(RtParams), P(C.c_double), P(C.c_ubyte), P(RtStats)],
                            C.c_int),
        "rt_render_devices": ([P(RtSphere), C.c_int, P(RtCamera), P(RtParams), P(C.c_int),
                               C.c_int, P(C.c_double), P(C.c_ubyte), P(RtStats)], C.c_int),
        "rt_host_alloc": ([C.c_size_t, P(C.c_void_p)], C.c_int),
        "rt_host_free": ([C.c_void_p], C.c_int),
        "rt_host_register": ([C.c_void_p, C.c_size_t], C.c_int),
        "rt_host_unregister": ([C.c_void_p], C.c_int),
        "rt_context_set_row_pitch": ([C.c_void_p, C.c_size_t, C.c_size_t], C.c_int),
        "rt_context_wait_drain": ([C.c_void_p, C.c_void_p], C.c_int),
    }
    for name, (args, res) in sig.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    if L.rt_abi_version() != ABI_VERSION:
        raise RtError(f"{lib_path}: ABI version {L.rt_abi_version()}, this binding is "
                      f"{ABI_VERSION} (include/rt.h RT_ABI_VERSION)")
    _lib = L
    return L


def check(rc: int, what: str) -> None:
    if rc != RT_OK:
        msg = load().rt_last_error().decode(errors="replace")
        raise RtError(f"{what} failed: {ERRORS.get(rc, rc)}: {msg}")
