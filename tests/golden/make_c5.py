"""Generate tests/golden/c5_pixels.json from the REFERENCE ITSELF: sampled
pixels of C5 (the final scene, 1200x800 at 10000 spp, depth 50, seed 0) at
full spp, each rendered by the reference's own pixel loop (oracle/_ref/
ref_render: programs/*.cc compiled unmodified, counter RNG interposed).

    python tests/golden/make_c5.py        # ~1 min on 8 cores (build container)
"""
from __future__ import annotations

import json
import os
import sys
import tempfile
from concurrent.futures import ThreadPoolExecutor

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

import oracle as O  # noqa: E402

W, H, SPP, N = 1200, 800, 10000, 8


def main() -> None:
    rng = np.random.default_rng(5005)
    ii = rng.integers(0, W, N).tolist()
    rr = rng.integers(0, H, N).tolist()  # output rows (0 = top)

    def one(k):
        i, r = ii[k], rr[k]
        with tempfile.TemporaryDirectory() as td:
            a = os.path.join(td, "a.bin")
            _, st = O.run_ref(["--scene", "final", "--width", str(W), "--height", str(H),
                               "--spp", str(SPP), "--seed", "0", "--rows", f"{r}:{H}:1",
                               "--cols", f"{i}:{i + 1}", "--accum", a])
            px = np.fromfile(a, dtype=np.float64).reshape(3)
        return dict(i=i, row=r, accum=[float(v).hex() for v in px], rays=st.get("rays"))

    with ThreadPoolExecutor(8) as ex:
        pix = list(ex.map(one, range(N)))
    cam = O.camera_look_at(aspect=W / H)
    out = dict(width=W, height=H, spp=SPP, max_depth=50, seed=0,
               camera=[[float(v).hex() for v in row] for row in cam], pixels=pix,
               source="oracle/_ref/ref_render (the reference sources), one process per pixel")
    with open(os.path.join(HERE, "c5_pixels.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(N, "pixels written")


if __name__ == "__main__":
    main()
