"""MI355X-native path-tracing hot path of fengye/PeterShirleyRaytracer.

The product is ``lib/libpsrt.so`` (HIP kernels for gfx950 behind the C ABI in
``include/rt.h``) plus the C++ host (``csrc/host``, ``include/raytracer``).
This Python package is host plumbing over that C ABI: scene/camera helpers,
one-shot and device-resident renders, PPM output, and the multi-GPU sharding
used by ``bench.py``. See DESIGN.md.
"""
from .render import (Context, DeviceGroup, LensCamera, SceneFile, camera_default, camera_look_at,
                     camera_look_at_lens, device_count, format_scene, host_array, load_scene, params,
                     parse_scene, ppm_p3, probe_f64, quantize, render, render_devices,
                     render_materials,
                     rows_owned, save_scene, scene_book_final, scene_random_spheres,
                     scene_two_spheres, get_tuning, set_tuning, tuning, write_ppm)

__all__ = [
    "Context", "DeviceGroup", "LensCamera", "SceneFile", "camera_default", "camera_look_at",
    "camera_look_at_lens", "device_count", "format_scene", "host_array", "load_scene", "params", "parse_scene",
    "ppm_p3", "probe_f64", "quantize", "render", "render_devices", "render_materials", "rows_owned", "save_scene",
    "scene_book_final", "scene_random_spheres", "scene_two_spheres", "get_tuning", "set_tuning",
    "tuning", "write_ppm",
]
