"""Host-buffer rate of the drop-in C ABI (rt_render: the frame's FP64 sums
and PPM bytes land in host memory, so every frame crosses PCIe), next to the
device-resident rate bench.py reports. C3 by default.

    python scripts/host_path.py [--frames 10] [--config c3]
"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import petershirleyraytracer_amd as P  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--frames", type=int, default=10)
ap.add_argument("--config", default="c3", choices=("c2", "c3", "c4"))
ap.add_argument("--group", type=int, default=0,
                help="render through rt_render_devices with this many members on device 0")
ap.add_argument("--rows", default="", help="R/G: only rows R, R+G, ... (a C4 row band: 0/8)")
ap.add_argument("--out", default="new", choices=("new", "reuse", "pinned", "pinned-bytes"),
                help="outputs: new arrays per frame (pageable, first touch), the same pageable "
                     "arrays every frame, page-locked arrays (host_array) every frame, or the "
                     "write_color bytes alone in a page-locked array (what main() prints)")
args = ap.parse_args()
w, h, spp = 1200, 800, 100
if args.config == "c4":
    w, h, spp = 3840, 2160, 500
if args.config == "c2":
    sph, cam = P.scene_two_spheres(), P.camera_default()
else:
    sph, cam = P.scene_random_spheres(1), P.camera_look_at(aspect=w / h)
r0, g0 = (int(x) for x in args.rows.split("/")) if args.rows else (0, 1)
shape = (P.rows_owned(h, r0, g0), w, 3)
out = None
if args.out == "reuse":
    out = (np.zeros(shape), np.zeros(shape, np.uint8))
elif args.out == "pinned":
    out = (P.host_array(shape), P.host_array(shape, np.uint8))
elif args.out == "pinned-bytes":
    out = (None, P.host_array(shape, np.uint8))
if args.group:
    grp = P.DeviceGroup([0] * args.group)
    grp.set_scene(sph, cam)
    one = lambda: grp.render(w, h, spp, row_offset=r0, row_stride=g0, out=out)  # noqa: E731
else:
    one = lambda: P.render(sph, cam, w, h, spp, row_offset=r0, row_stride=g0, out=out)  # noqa: E731
one()  # warm-up: context(s), scene structures, camera lists
ts, ks = [], []
for _ in range(args.frames):
    t0 = time.perf_counter()
    acc, rgb, st = one()
    ts.append(time.perf_counter() - t0)
    ks.append(st["kernel_ms"])
ms = 1e3 * sum(ts) / len(ts)
print({"config": args.config, "rows": args.rows or "all", "group_members": args.group,
       "outputs": args.out,
       "frames": args.frames, "ms_per_frame_host_buffers": round(ms, 3),
       "msamples_per_s_host_buffers": round(shape[0] * w * spp / (ms * 1e-3) / 1e6, 1),
       "psrt_trace_ms": round(sum(ks) / len(ks), 3),
       "host_bytes_per_frame": int((acc.nbytes if acc is not None else 0) + rgb.nbytes)})
