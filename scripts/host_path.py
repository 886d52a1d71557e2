"""Host-buffer rate of the drop-in C ABI (rt_render: the frame's FP64 sums
and PPM bytes land in host memory, so every frame crosses PCIe), next to the
device-resident rate bench.py reports. C3 by default.

    python scripts/host_path.py [--frames 10] [--config c3]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import petershirleyraytracer_amd as P  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--frames", type=int, default=10)
ap.add_argument("--config", default="c3", choices=("c2", "c3"))
args = ap.parse_args()
w, h, spp = 1200, 800, 100
if args.config == "c2":
    sph, cam = P.scene_two_spheres(), P.camera_default()
else:
    sph, cam = P.scene_random_spheres(1), P.camera_look_at(aspect=w / h)
P.render(sph, cam, w, h, spp)  # warm-up: context, scene structures, camera lists
ts, ks = [], []
for _ in range(args.frames):
    t0 = time.perf_counter()
    acc, rgb, st = P.render(sph, cam, w, h, spp)
    ts.append(time.perf_counter() - t0)
    ks.append(st["kernel_ms"])
ms = 1e3 * sum(ts) / len(ts)
print({"config": args.config, "frames": args.frames, "ms_per_frame_host_buffers": round(ms, 3),
       "msamples_per_s_host_buffers": round(w * h * spp / (ms * 1e-3) / 1e6, 1),
       "psrt_trace_ms": round(sum(ks) / len(ks), 3),
       "host_bytes_per_frame": int(acc.nbytes + rgb.nbytes)})
