"""Two C3 frames on two contexts (two streams / hardware queues): one after
the other vs enqueued together (their persistent launches then share the
CUs). Prints ms per frame for both; PSRT_LIB selects the library build."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import petershirleyraytracer_amd as P  # noqa: E402

sph = P.scene_random_spheres(1)
cam = P.camera_look_at(aspect=1.5)
ctxs = [P.Context(0) for _ in range(2)]
for c in ctxs:
    c.set_scene(sph, cam)
bufs = [(torch.zeros((800, 1200, 3), dtype=torch.float64, device="cuda:0"),
         torch.zeros((800, 1200, 3), dtype=torch.uint8, device="cuda:0")) for _ in ctxs]
prm = P.params(1200, 800, 100)


def render(k):
    ctxs[k].render_device(prm, bufs[k][0].data_ptr(), bufs[k][1].data_ptr(), ctxs[k].stream())


def run(mode, reps=int(os.environ.get("REPS", "5"))):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        if mode == "seq":
            render(0)
            ctxs[0].sync_stats()
            render(1)
            ctxs[1].sync_stats()
        else:
            render(0)
            render(1)
            ctxs[0].sync_stats()
            ctxs[1].sync_stats()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / (2 * reps) * 1e3


run("seq", 1)
for m in ("seq", "conc", "seq", "conc"):
    print(os.environ.get("PSRT_LIB", "default").split("/")[-1], m, round(run(m), 3), flush=True)
