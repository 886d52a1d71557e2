"""Diagnostic (the stamps tuning knob): the wave timeline (start, queue-empty and
exit times over waves) of a C3 shard launch of 1 and of 20 frames.

  python3 scripts/stamps_shard.py R G
"""
import os
import sys

sys.path.insert(0, ".")
import torch  # noqa: E402

import petershirleyraytracer_amd as P  # noqa: E402

r, g = int(sys.argv[1]), int(sys.argv[2])
ctx = P.Context(0)
ctx.set_scene(P.scene_random_spheres(1), P.camera_look_at(aspect=1.5))
rows = len(range(r, 800, g))
acc = torch.zeros((20, rows, 1200, 3), dtype=torch.float64, device="cuda:0")
s = torch.cuda.current_stream().cuda_stream
prm = P.params(1200, 800, 100, 50, 0, r, g, 0)
ptr = [acc[f].data_ptr() for f in range(20)]
for nb in (1, 20, 1, 20):
    ctx.render_device_frames(prm, nb, ptr[:nb], None, s)
    ctx.sync_stats()
ctx.set_tuning("stamps", 1)  # the diagnostic kernel variant (include/rt.h tuning knobs)
for nb in (1, 20):
    ctx.render_device_frames(prm, nb, ptr[:nb], None, s)
    st = ctx.sync_stats()
    print(f"frames {nb}: kernel_ms {st['kernel_ms']:.3f}", file=sys.stderr, flush=True)
