"""Throughput of the materials extension: the book's final scene
(rt_scene_book_final, lens camera: aperture 0.1, focus 10, vfov 20, 3:2) at
W x H x spp, max depth 50, on one GPU, with the C restatement timed on the
host cores beside it (a bounded sample of rows).

    python scripts/bench_materials.py [--width 1200 --height 800 --spp 10 --steps 10]

Prints one JSON line. Frames are device-resident (no D2H in the timed region).
`value` is the rate of the timed frames in launches of --batch frames
(rt_render_device_frames; 0 = auto: all timed frames in one launch, <= 32),
as bench.py's headline; `unbatched` is the same frames one per launch. The
roofline counts what the counting variant executed, with bench.py's issue
weights (WEIGHTS: measured instruction costs, scripts/isa_rates.hip).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=1200)
    ap.add_argument("--height", type=int, default=800)
    ap.add_argument("--spp", type=int, default=10)
    ap.add_argument("--depth", type=int, default=50)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--cpu-rows", type=int, default=8)
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--no-cull", action="store_true")
    ap.add_argument("--tune", default="",
                    help="measurement knobs (include/rt.h rt_context_set_tuning), name=value[,...]")
    ap.add_argument("--batch", type=int, default=0,
                    help="frames per trace launch (<= 32; 0 = all timed frames, 1 = one per launch)")
    a = ap.parse_args()

    import torch
    import petershirleyraytracer_amd as P
    from petershirleyraytracer_amd.render import FLAG_CULL_STATS, FLAG_MATERIALS, FLAG_NO_CULL

    for kv in filter(None, a.tune.split(",")):
        k, v = kv.split("=")
        P.set_tuning(k.strip(), float(v))
    W, H, S = a.width, a.height, a.spp
    sp, mt = P.scene_book_final(1)
    lens = P.camera_look_at_lens(aspect=W / H)
    ctx = P.Context(0)
    ctx.set_scene(sp, lens.base)
    ctx.set_materials(mt, lens)
    acc = torch.zeros((H, W, 3), dtype=torch.float64, device="cuda")
    rgb = torch.zeros((H, W, 3), dtype=torch.uint8, device="cuda")
    flags = FLAG_MATERIALS | (FLAG_NO_CULL if a.no_cull else 0)
    st = ctx.stream()
    B = min(32, a.steps) if a.batch <= 0 else min(32, a.batch)
    accs = [torch.zeros((H, W, 3), dtype=torch.float64, device="cuda") for _ in range(max(1, B))]
    for i in range(a.warmup):
        ctx.render_device(P.params(W, H, S, a.depth, 100 + i, flags=flags), acc.data_ptr(),
                          rgb.data_ptr(), st)
        ctx.sync_stats()
    if B > 1:  # the sample buffer grows to B frames outside the timed region
        ctx.render_device_frames(P.params(W, H, S, a.depth, 200, flags=flags), B,
                                 [x.data_ptr() for x in accs], None, st)
        ctx.sync_stats()

    def timed(b):
        """a.steps frames (seeds 0..) in launches of up to b frames"""
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        kms, rays, f0 = 0.0, 0, 0
        while f0 < a.steps:
            nb = min(b, a.steps - f0)
            if nb == 1:
                ctx.render_device(P.params(W, H, S, a.depth, f0, flags=flags), acc.data_ptr(),
                                  rgb.data_ptr(), st)
            else:
                ctx.render_device_frames(P.params(W, H, S, a.depth, f0, flags=flags), nb,
                                         [x.data_ptr() for x in accs[:nb]], None, st)
            s = ctx.sync_stats()
            kms += s["kernel_ms"]
            rays += s["rays"]
            f0 += nb
        return (time.perf_counter() - t0) * 1e3 / a.steps, kms / a.steps, rays

    step, kms, rays = timed(B)
    unbatched = None
    if B > 1:
        s1, k1, _ = timed(1)
        unbatched = {"ms_per_step": round(s1, 4), "value": round(W * H * S / (s1 * 1e3), 2),
                     "kernel_ms": round(k1, 4)}
    # one untimed frame of the counting variant: the sphere / box tests the
    # kernel executes (deterministic: the same for every frame of a seed)
    ctx.render_device(P.params(W, H, S, a.depth, 0, flags=flags | FLAG_CULL_STATS),
                      acc.data_ptr(), rgb.data_ptr(), st)
    cs = ctx.sync_stats()
    # FP64-op slots as bench.py counts them for psrt_trace (WEIGHTS: every
    # sphere test of this kernel is a full FP64 one, there is no pre-reject)
    from bench import SHADE_OPS_PER_RAY, WEIGHTS
    ops = (cs["tests_executed"] * WEIGHTS["full_sphere_test"] + cs["box_tests"] * WEIGHTS["box_test"]
           + cs["root_box_tests"] * WEIGHTS["root_box_test"] + cs["rays"] * SHADE_OPS_PER_RAY)
    achieved = ops / (kms * 1e-3) / 1e12
    roof = {"bound": "valu", "achieved": round(achieved, 4), "peak": 39.32, "unit": "TFLOP/s",
            "frac": round(achieved / 39.32, 4), "traffic": None, "kernel": "psrt_trace_mat",
            "avg_launch_ms": round(kms, 4), "full_sphere_tests_per_launch": cs["tests_executed"],
            "box_tests_evaluated_per_launch": cs["box_tests"],
            "root_box_tests_per_launch": cs["root_box_tests"], "rays_per_launch": cs["rays"],
            "issue_weights_fp64_slots": {k: round(v, 3) for k, v in WEIGHTS.items()},
            "note": "FP64-op slots (full FP64 sphere tests, FP32 slab tests and FP64 root-box "
                    "tests executed, each x its issue weight, + rays x 61) / kernel time per "
                    "frame, against 256 CU x 64 lanes x 2.4 GHz non-FMA FP64"}
    pmc = os.path.join(ROOT, "profiles", "pmc_mat.json")
    if os.path.exists(pmc):
        d = json.load(open(pmc))
        roof["valu_issue"] = {"simd_cycles_per_valu_inst": round(d.get("simd_cycles_per_valu", 0), 3),
                              "wait_inst_frac": round(d.get("wait_inst_frac", 0), 3),
                              "source": "profiles/pmc_mat.json"}
        if d.get("hbm_bytes_per_launch"):
            # FETCH_SIZE x 2 + WRITE_SIZE per one-frame PMC dispatch (KiB-corrected)
            roof["traffic"] = d["hbm_bytes_per_launch"]
            roof["traffic_note"] = ("HBM bytes per frame from the PMC passes (profiles/pmc_mat.json); "
                                    "algorithmic: 24 B colour record per sample written, read once "
                                    "by psrt_reduce_rgb")
    out = {
        "metric": "Msamples/sec (materials extension, book final scene)",
        "value": W * H * S / (step * 1e3),
        "unit": "Msamples/s",
        "ms_per_step": step,
        "kernel_ms": kms,
        "grays_per_s": rays / (step * a.steps * 1e6),
        "rays_per_sample": rays / (a.steps * W * H * S),
        "config": {"scene": "book_final(seed 1), 487 spheres, lambertian/metal/dielectric",
                   "width": W, "height": H, "spp": S, "max_depth": a.depth,
                   "lens": "aperture 0.1, focus 10", "cull": not a.no_cull,
                   **({"tune": a.tune} if a.tune else {})},
        "steps": a.steps, "warmup": a.warmup, "dtype": "f64", "roofline": roof,
        "frames_per_launch": B, "unbatched": unbatched,
    }
    ctx.close()
    # the C restatement on the host cores (the usable ones: affinity capped by
    # the cgroup CPU quota), a bounded sample of rows; then one thread
    import oracle
    from bench import host_cpus
    hc = host_cpus()
    threads = a.cpu_threads or hc["usable"]
    ol = oracle.camera_look_at_lens(aspect=W / H)
    osp, omt = oracle.scene_book_final(1)
    rows = a.cpu_rows
    t0 = time.perf_counter()
    _, crays = oracle.render_mat(osp, omt, ol, W, H, S, a.depth, 0, 0, max(1, H // rows),
                                 threads=threads)
    dt = time.perf_counter() - t0
    n = oracle.rows_owned(H, 0, max(1, H // rows)) * W * S
    t0 = time.perf_counter()
    oracle.render_mat(osp, omt, ol, W, H, S, a.depth, 0, H // 2, H, threads=1)
    dt1 = time.perf_counter() - t0
    out["cpu_baseline"] = {"value": n / (dt * 1e6), "unit": "Msamples/s", "cores": threads,
                           "kind": "port", "one_thread_value": W * S / (dt1 * 1e6),
                           "nproc": hc["nproc"], "cgroup_cpu_quota": hc["cgroup_quota"],
                           "cpu_model": hc["cpu_model"],
                           "sample": f"{n} samples ({n // (W * S)} rows, C restatement "
                                     f"oracle/rt_oracle_mat.c, {threads} threads); one thread: "
                                     f"the middle row"}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
