"""Kernel time of the same C3 frame rendered one at a time on N contexts (each
its own stream / HIP hardware queue): does the queue a launch lands on
matter? Prints per-context psrt_trace ms."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import petershirleyraytracer_amd as P  # noqa: E402

n = int(os.environ.get("NCTX", "4"))
rounds = int(os.environ.get("ROUNDS", "4"))
sph = P.scene_random_spheres(1)
cam = P.camera_look_at(aspect=1.5)
ctxs = []
for _ in range(n):
    c = P.Context(0)
    c.set_scene(sph, cam)
    ctxs.append(c)
acc = torch.zeros((800, 1200, 3), dtype=torch.float64, device="cuda:0")
rgb = torch.zeros((800, 1200, 3), dtype=torch.uint8, device="cuda:0")
prm = P.params(1200, 800, 100)
res = {k: [] for k in range(n)}
for r in range(rounds):
    for k, c in enumerate(ctxs):
        c.render_device(prm, acc.data_ptr(), rgb.data_ptr(), c.stream())
        st = c.sync_stats()
        torch.cuda.synchronize()
        res[k].append(round(st["kernel_ms"], 3))
for k in range(n):
    print("context", k, "kernel ms", res[k], flush=True)
