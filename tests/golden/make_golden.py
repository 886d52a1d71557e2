"""Generate the golden fixtures in tests/golden/ from the REFERENCE ITSELF.

Run in the build container (needs /root/reference and oracle/_ref/ref_render,
which `make -C oracle` builds from the reference sources). Every expected value
below comes out of the reference's own code (programs/*.cc, *.h compiled
unmodified, driven by oracle/ref_driver.cc); the oracle restatement is only
cross-checked here, never used as the source of an expected value — except
trace_kat.json (per-bounce records the reference cannot print), written by
the oracle only after the oracle is shown bit-equal to the reference on the
same scenes.

    python tests/golden/make_golden.py            # small fixtures (~1 min)
    python tests/golden/make_golden.py --large    # + full-size checksums (C2, C3; ~10 min on 8 cores)
"""
from __future__ import annotations

import hashlib
import json
import os
import subprocess
import sys
import tempfile
from concurrent.futures import ThreadPoolExecutor

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

import oracle as O  # noqa: E402


def hx(x: float) -> str:
    return float(x).hex()


def ref_render(args, rows_total, width, procs=1):
    """Run the reference pixel loop, optionally over `procs` interleaved row
    shards in parallel; returns (accum[rows, W, 3], ppm P3 bytes, rays)."""
    with tempfile.TemporaryDirectory() as td:
        def one(k):
            acc = os.path.join(td, f"a{k}.bin")
            extra = ["--rows", f"{k}:{procs}"] if procs > 1 else []
            _, st = O.run_ref([*args, *extra, "--accum", acc, "--ppm", os.path.join(td, f"p{k}.ppm")])
            rows = len(range(k, rows_total, procs))
            # the reference's own write_color text (color.h:21-23), one line per pixel
            body = open(os.path.join(td, f"p{k}.ppm")).read().split("\n", 3)[3]
            lines = body.splitlines()
            assert len(lines) == rows * width
            return (np.fromfile(acc, dtype=np.float64).reshape(rows, width, 3), st["rays"],
                    [lines[r * width:(r + 1) * width] for r in range(rows)])
        with ThreadPoolExecutor(procs) as ex:
            parts = list(ex.map(one, range(procs)))
    accum = np.zeros((rows_total, width, 3), dtype=np.float64)
    text_rows = [None] * rows_total
    for k, (a, _, tr) in enumerate(parts):
        accum[k::procs] = a
        text_rows[k::procs] = tr
    rays = sum(r for _, r, _ in parts)
    # The PPM is the reference's own text (main.cc:70 header + write_color
    # lines of the shards, re-interleaved); the oracle's quantizer must
    # reproduce it byte for byte (that pins oracle.quantize / ppm_p3 directly).
    ppm = (f"P3\n{width} {rows_total}\n255\n" + "".join(
        "".join(l + "\n" for l in row) for row in text_rows)).encode()
    spp = int(args[args.index("--spp") + 1])
    assert ppm == O.ppm_p3(O.quantize(accum, spp)), "oracle quantizer differs from write_color"
    return accum, ppm, rays


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a, dtype=np.float64).tobytes()).hexdigest()


def main(large: bool) -> None:
    assert O.have_ref(), "build oracle/_ref/ref_render first: make -C oracle"
    out = {}

    # 1. glibc stream: the reference main() as shipped (RNG scaling fixed)
    ref_main, _ = O.run_ref(["--reference-main"])
    out["reference_main_p3_md5"] = hashlib.md5(ref_main).hexdigest()
    g10, _ = O.run_ref(["--rng", "glibc", "--spp", "10"])
    out["glibc_two_400x225x10_p3_md5"] = hashlib.md5(g10).hexdigest()
    with open(os.path.join(HERE, "reference_glibc.json"), "w") as f:
        json.dump(out, f, indent=1)

    # 2. counter stream, two-sphere world (main.cc:61-63), default camera
    two = O.scene_two_spheres()
    cam16x9 = O.camera_default()
    fx = {"scene": "two", "camera": [[hx(v) for v in row] for row in cam16x9],
          "spheres": [[hx(v) for v in s] for s in two], "cases": []}
    for (w, h, spp, depth, seed, rows_spec) in [
        (64, 36, 10, 50, 0, None), (400, 225, 10, 50, 0, None), (400, 225, 100, 50, 0, None),
        (64, 36, 7, 5, 12345, None), (64, 36, 3, 0, 7, None), (64, 36, 3, -1, 7, None),
        (400, 225, 10, 50, 0, (1, 3)),
    ]:
        args = ["--scene", "two", "--width", str(w), "--height", str(h), "--spp", str(spp),
                "--depth", str(depth), "--seed", str(seed)]
        if rows_spec:
            args += ["--rows", f"{rows_spec[0]}:{rows_spec[1]}"]
        rows = len(range(rows_spec[0], h, rows_spec[1])) if rows_spec else h
        acc, ppm, rays = ref_render(args, rows, w, procs=1 if rows_spec else min(8, rows))
        # cross-check: the oracle restatement reproduces the reference bit for bit
        oacc, _, orays = O.render(two, cam16x9, w, h, spp, depth, seed,
                                  *(rows_spec or (0, 1)), threads=8)
        assert np.array_equal(oacc.view(np.uint64), acc.view(np.uint64)), (w, h, spp, depth)
        assert orays == rays
        case = dict(width=w, height=h, spp=spp, max_depth=depth, seed=seed,
                    row_offset=rows_spec[0] if rows_spec else 0,
                    row_stride=rows_spec[1] if rows_spec else 1,
                    accum_sha256=sha(acc), p3_md5=hashlib.md5(ppm).hexdigest(), rays=rays)
        if w * rows <= 64 * 36:
            name = f"counter_two_{w}x{h}x{spp}_d{depth}_s{seed}.npy"
            np.save(os.path.join(HERE, name), acc)
            case["accum_npy"] = name
        fx["cases"].append(case)
        print("two", case["width"], case["height"], case["spp"], case["max_depth"], "ok", flush=True)
    with open(os.path.join(HERE, "counter_two.json"), "w") as f:
        json.dump(fx, f, indent=1)

    # 3. final random-spheres scene (reference vec3/sphere/random_double)
    with tempfile.TemporaryDirectory() as td:
        dump = os.path.join(td, "s.txt")
        subprocess.run([O.REF_BIN, "--scene", "final", "--width", "1200", "--height", "800",
                        "--rows", "0:1:0", "--dump-scene", dump], check=True, capture_output=True)
        lines = open(dump).read().split("\n")
    n = int(lines[0].split()[1])
    spheres = np.array([[float.fromhex(v) for v in ln.split()] for ln in lines[1:1 + n]])
    cam = np.array([[float.fromhex(v) for v in ln.split()] for ln in lines[2 + n:6 + n]])
    assert np.array_equal(spheres, O.scene_random_spheres(1))
    assert np.array_equal(cam, O.camera_look_at(aspect=1200 / 800))
    ff = {"scene": "final", "scene_seed": 1, "n": n,
          "spheres": [[hx(v) for v in s] for s in spheres],
          "camera_1200x800": [[hx(v) for v in row] for row in cam], "cases": []}
    for (w, h, spp, seed) in [(48, 32, 4, 0), (120, 80, 8, 0)]:
        args = ["--scene", "final", "--width", str(w), "--height", str(h), "--spp", str(spp),
                "--seed", str(seed)]
        acc, ppm, rays = ref_render(args, h, w, procs=8)
        cam_wh = O.camera_look_at(aspect=w / h)
        oacc, _, orays = O.render(spheres, cam_wh, w, h, spp, 50, seed, threads=8)
        assert np.array_equal(oacc.view(np.uint64), acc.view(np.uint64)), (w, h, spp)
        case = dict(width=w, height=h, spp=spp, max_depth=50, seed=seed,
                    camera=[[hx(v) for v in row] for row in cam_wh],
                    accum_sha256=sha(acc), p3_md5=hashlib.md5(ppm).hexdigest(), rays=rays)
        if w * h <= 48 * 32:
            name = f"counter_final_{w}x{h}x{spp}.npy"
            np.save(os.path.join(HERE, name), acc)
            case["accum_npy"] = name
        ff["cases"].append(case)
        print("final", w, h, spp, "ok", flush=True)

    # 3b. sampled pixels of the big configs (full spp, reference pixel loop)
    rng = np.random.default_rng(2024)
    ff["sampled"] = []
    for (w, h, spp, nsamp) in [(1200, 800, 100, 24), (3840, 2160, 500, 8)]:
        cam_wh = O.camera_look_at(aspect=w / h)
        ii = rng.integers(0, w, nsamp)
        rr = rng.integers(0, h, nsamp)  # output rows (0 = top)
        pix = []
        for i, r in zip(ii.tolist(), rr.tolist()):
            args = ["--scene", "final", "--width", str(w), "--height", str(h), "--spp", str(spp),
                    "--seed", "0", "--rows", f"{r}:{h}:1", "--cols", f"{i}:{i + 1}"]
            with tempfile.TemporaryDirectory() as td:
                a = os.path.join(td, "a.bin")
                O.run_ref([*args, "--accum", a])
                px = np.fromfile(a, dtype=np.float64).reshape(3)
            pix.append(dict(i=i, row=r, accum=[hx(v) for v in px]))
            print("sampled", w, h, i, r, flush=True)
        ff["sampled"].append(dict(width=w, height=h, spp=spp, max_depth=50, seed=0,
                                  camera=[[hx(v) for v in row] for row in cam_wh], pixels=pix))
    with open(os.path.join(HERE, "counter_final.json"), "w") as f:
        json.dump(ff, f, indent=1)

    # 4. sphere::hit / hittable_list::hit known answers (reference --kat)
    cases = kat_cases(spheres)
    with tempfile.TemporaryDirectory() as td:
        p = os.path.join(td, "k.txt")
        with open(p, "w") as f:
            for c in cases:
                f.write(" ".join([str(len(c["spheres"]))] +
                                 [hx(v) for s in c["spheres"] for v in s] +
                                 [hx(v) for v in c["o"]] + [hx(v) for v in c["d"]] +
                                 [hx(c["tmin"]), hx(c["tmax"])]) + "\n")
        res = subprocess.run([O.REF_BIN, "--kat", p], check=True, capture_output=True).stdout
    fs = spheres.tolist()
    for c, line in zip(cases, res.decode().strip().split("\n")):
        toks = line.split()
        c["expect_index"] = int(toks[0])
        c["expect"] = toks[1:]
        # the final scene's list is stored once, in counter_final.json
        c["spheres"] = "final" if c["spheres"] == fs else [[hx(v) for v in s] for s in c["spheres"]]
        c["o"] = [hx(v) for v in c["o"]]
        c["d"] = [hx(v) for v in c["d"]]
        c["tmin"], c["tmax"] = hx(c["tmin"]), hx(c["tmax"])
    with open(os.path.join(HERE, "kat_hit.json"), "w") as f:
        json.dump(cases, f, indent=0)

    # 5. RNG known answers: glibc rand() itself, and the counter-stream spec
    import ctypes
    libc = ctypes.CDLL("libc.so.6")
    rk = {"glibc": [], "counter": []}
    for seed in (1, 42, 2147483646):
        libc.srand(seed)
        rk["glibc"].append(dict(seed=seed, draws=[libc.rand() for _ in range(64)]))
    for (seed, pixel, sample) in [(0, 0, 0), (0, 89999, 9), (1, 12345, 0), (2**63 + 5, 4000000, 9999)]:
        rk["counter"].append(dict(seed=str(seed), pixel=pixel, sample=sample,
                                  draws=O.counter_draws(seed, pixel, sample, 32).tolist()))
    with open(os.path.join(HERE, "rng_kat.json"), "w") as f:
        json.dump(rk, f, indent=0)

    # 6. per-bounce path traces (oracle, validated bit-equal above)
    tk = []
    for (sc_name, sc, cam_a, w, h) in [("two", two, cam16x9, 400, 225),
                                       ("final", spheres, O.camera_look_at(aspect=1.5), 1200, 800)]:
        for (i, j, s) in [(200, 112, 0), (10, 5, 3), (399, 0, 9), (123, 45, 1), (57, 100, 2),
                          (300, 150, 4), (0, 224, 5), (250, 60, 8)]:
            col, bounces = O.trace_sample(sc, cam_a, w, h, i, j, s)
            tk.append(dict(scene=sc_name, width=w, height=h, i=i, j=j, s=s,
                           color=[hx(v) for v in col],
                           bounces=[dict(o=[hx(v) for v in b["o"]], d=[hx(v) for v in b["d"]],
                                         t=hx(b["t"]), index=b["index"],
                                         front_face=b["front_face"],
                                         draws_after=b["draws_after"]) for b in bounces]))
    with open(os.path.join(HERE, "trace_kat.json"), "w") as f:
        json.dump(tk, f, indent=0)

    if large:
        large_fixtures(two, cam16x9, spheres)


def kat_cases(final_spheres):
    inf = float("inf")
    S = [0.0, 0.0, -1.0, 0.5]
    cases = [
        dict(name="tangent", spheres=[S], o=[0.5, 0, 0], d=[0, 0, -1], tmin=0.0, tmax=inf),
        dict(name="miss", spheres=[S], o=[0.6, 0, 0], d=[0, 0, -1], tmin=0.0, tmax=inf),
        dict(name="inside_far_root", spheres=[S], o=[0, 0, -1], d=[1, 0, 0], tmin=0.0, tmax=inf),
        dict(name="t_eq_tmin_zero", spheres=[S], o=[0, 0, -0.5], d=[0, 0, 1], tmin=0.0, tmax=inf),
        dict(name="t_eq_tmax", spheres=[S], o=[0, 0, 0], d=[0, 0, -1], tmin=0.0, tmax=0.5),
        dict(name="beyond_tmax", spheres=[S], o=[0, 0, 0], d=[0, 0, -1], tmin=0.0, tmax=0.4999),
        dict(name="behind", spheres=[S], o=[0, 0, 0], d=[0, 0, 1], tmin=0.0, tmax=inf),
        dict(name="tie_later_wins", spheres=[[0, 0, -2, 1.0], [1, 0, -1, 1.0]], o=[0, 0, 0],
             d=[0, 0, -1], tmin=0.0, tmax=inf),
        dict(name="tie_later_wins_rev", spheres=[[1, 0, -1, 1.0], [0, 0, -2, 1.0]], o=[0, 0, 0],
             d=[0, 0, -1], tmin=0.0, tmax=inf),
        dict(name="nearer_first", spheres=[[0, 0, -3, 1.0], [0, 0, -5, 1.0]], o=[0, 0, 0],
             d=[0, 0, -1], tmin=0.0, tmax=inf),
        dict(name="unnormalised_dir", spheres=[S], o=[0, 0, 0], d=[0, 0, -3], tmin=0.0, tmax=inf),
        dict(name="zero_dir_nan", spheres=[S], o=[0, 0, 0], d=[0, 0, 0], tmin=0.0, tmax=inf),
        dict(name="ground_graze", spheres=[[0, -100.5, 0, 100.0]], o=[0, 0, 0],
             d=[0, -0.005, -1], tmin=0.0, tmax=inf),
        dict(name="two_sphere_world", spheres=[S, [0, -100.5, 0, 100.0]], o=[0, 0, 0],
             d=[0.1, -0.3, -1], tmin=0.0, tmax=inf),
    ]
    rng = np.random.default_rng(7)
    fs = final_spheres.tolist()
    for k in range(48):
        # random rays from random points on random spheres (self-intersection regime)
        si = int(rng.integers(0, len(fs)))
        c = np.array(fs[si][:3])
        r = fs[si][3]
        v = rng.normal(size=3)
        v /= np.linalg.norm(v)
        o = (c + r * v).tolist()
        d = rng.normal(size=3).tolist()
        cases.append(dict(name=f"final_random_{k}", spheres=fs, o=o, d=d, tmin=0.0, tmax=inf))
    return cases


def large_fixtures(two, cam16x9, spheres):
    """Full-size frame checksums (C2 and C3 of SURVEY.md §8a) from the reference."""
    path = os.path.join(HERE, "large.json")
    big = json.load(open(path)) if os.path.exists(path) else {}
    for (name, args, rows, w) in [
        ("two_1200x800x100", ["--scene", "two", "--width", "1200", "--height", "800",
                              "--spp", "100"], 800, 1200),
        ("final_1200x800x100", ["--scene", "final", "--width", "1200", "--height", "800",
                                "--spp", "100"], 800, 1200),
    ]:
        if name in big:
            continue
        acc, ppm, rays = ref_render(args, rows, w, procs=8)
        big[name] = dict(args=args, accum_sha256=sha(acc), p3_md5=hashlib.md5(ppm).hexdigest(),
                         rays=rays, mean_rgb8=float(O.quantize(acc, 100).mean()))
        with open(path, "w") as f:
            json.dump(big, f, indent=1)
        print("large", name, big[name], flush=True)


if __name__ == "__main__":
    main(large="--large" in sys.argv)
