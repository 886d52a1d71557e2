#!/usr/bin/env python3
"""Benchmark of the MI355X path-tracing hot path (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3]
    torchrun --nproc-per-node N bench.py --gpus N ...        (N > 1, RCCL)

A step is one full frame of the configured workload: every rank renders its
interleaved rows (psrt_camera_lists + psrt_trace + psrt_reduce through
rt_render_device, inputs resident in HBM) and quantises them (write_color,
color.h:8-24, per pixel); the uint8 rows are gathered to rank 0 over RCCL
(--gather-fp64: the FP64 accumulators, quantised on rank 0). Rank 0 prints
one JSON line; value = W*H*spp*K / wall, wall = max over ranks between
barriers.

Scaling (--scaling): "strong" (default) renders the configured frame itself
on any N, rows interleaved over the ranks: the BASELINE metric (W*H*spp/wall
at 1/2/4/8 GPUs) on one fixed workload. "weak" is an opt-in study that keeps
each GPU's work fixed: on N GPUs the frame is the configured W x H at N x spp
(config_id gets a "-weak" suffix, so its value is never read as the
configured frame's number).

The BASELINE's 8-GPU configuration (C4, 3840x2160x500) is
    torchrun --nproc-per-node 8 bench.py --gpus 8 --config c4
(strong, the default); the N=1 default stays C3 so BENCH and SCALE agree.

Each timed step ends with the frame's write_color bytes in pinned host memory
(a device-to-host copy of the rank-0 frame, main.cc:70,86: the reference's
loop ends by emitting the image). After the timed steps the timed kernel's own
output is checked: its frame of seed --seed against the reference itself
(oracle/_ref/ref_render) bit for bit on sampled pixels at the frame's full spp
(N = 1: the CPU baseline's rows, or a column window when spp > 100; N > 1: the
FP64 accumulators gathered to rank 0, every rank's rows covered), and the last
frame of the last timed launch against a one-frame render of its seed
(`batch_check`).

Default workload (BASELINE.json north star, configs[2]): the final
random-spheres scene (485 spheres), 1200x800, 100 spp, depth 50.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Msamples/sec (W×H×spp/wall) at 1/2/4/8 GPUs; PSNR vs CPU PPM"

CONFIGS = {
    "c1": dict(scene="two", width=400, height=225, spp=10,
               desc="two-sphere world (main.cc:61-63), 400x225, 10 spp, depth 50"),
    "c2": dict(scene="two", width=1200, height=800, spp=100,
               desc="two-sphere world (main.cc:61-63), 1200x800, 100 spp, depth 50"),
    "c3": dict(scene="final", width=1200, height=800, spp=100,
               desc="final random-spheres scene (485 spheres), 1200x800, 100 spp, depth 50"),
    "c4": dict(scene="final", width=3840, height=2160, spp=500,
               desc="final random-spheres scene (485 spheres), 3840x2160, 500 spp, depth 50"),
    "c5": dict(scene="final", width=1200, height=800, spp=10000,
               desc="final random-spheres scene (485 spheres), 1200x800, 10000 spp, depth 50"),
}

# MI355X peaks (/opt/skills/guides/MI355X_MICROARCH.md): 256 CUs at 2.4 GHz;
# FP64 vector = half the FP32 vector rate: 16 lanes/clk/SIMD x 4 SIMDs -> one
# non-FMA FP64 op per lane-slot: 256 * 64 * 2.4e9 = 39.3e12 op/s.
PEAK_FP64_OPS = 256 * 64 * 2.4e9
PEAK_HBM = 8.0e12
# sphere.cc:6-14 per ray-sphere test: amc (3), A (5), HALF_B (5), C (5 + r*r + sub = 7),
# discriminant (3) = 23 FP64 ops (the reference-equivalent figure).
OPS_PER_TEST = 23
# Algorithmic work of psrt_trace as executed, by the kind of test that ran
# (the counting variant's tallies, RT_FLAG_CULL_STATS), each weighted by its
# operations' measured issue cost in FP64-op slots: one slot = one FP64 add,
# 4.4 SIMD cycles per wave64 instruction (scripts/isa_rates.hip; the peak
# below counts one slot per lane per cycle). Costs (cycles): FP64 add / mul /
# min / max 4.4, FP64 compare 4.2, v_rcp_f64 16.3, FP32 add / sub 2.35, FP32
# mul / FMA / min / max / compare 4.25, cvt f64 -> f32 4.2. DESIGN.md §7.
#   full FP64 sphere test (sphere.cc:6-14 with A hoisted per ray and r*r per
#     sphere, the same values): 17 FP64 add/mul + 1 compare = 79.0 cycles
#   FP32 pre-reject (Pre32): 4 add/sub + 5 mul/FMA + 1 compare + 1 cvt = 39.1
#   FP32 slab test (slab_hit): 6 FMA + 10 min/max + 1 compare = 72.25
#   FP64 root-box test (root_box_entry): 3 x (compare, v_rcp_f64, 4 add/mul,
#     4 min/max) + 2 FP64 ops + compare = 180.3
ISA_CYCLES_PER_SLOT = 4.4
WEIGHTS = {"full_sphere_test": (17 * 4.4 + 4.2) / 4.4,
           "prereject": (4 * 2.35 + 5 * 4.25 + 4.25 + 4.2) / 4.4,
           "box_test": 17 * 4.25 / 4.4,
           "root_box_test": (3 * (4.2 + 16.3 + 8 * 4.4) + 2 * 4.4 + 4.2) / 4.4}
# FP64 ops per traced ray outside the sphere/box tests (estimate from the
# kernel source): hit record 18 (ray.h:25-28, sphere.cc:34-36, hittable.h:14-18),
# scatter 26 (vec3.h:102-109, main.cc:42-43, the new ray's A), look-ahead
# trials 9 x 1.91 per scatter (vec3.h:83-95) ~ 17  ->  ~61
SHADE_OPS_PER_RAY = 61
# one finished sample's record in HBM: t (FP64) + k (uint16) (psrt_kernels.h kSampleBytes)
SAMPLE_RECORD_BYTES = 10


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--max-depth", type=int, default=50)
    ap.add_argument("--cpu-seconds", type=float, default=12.0,
                    help="target CPU work of the bounded reference baseline sample")
    ap.add_argument("--cpu-procs", type=int, default=0,
                    help="reference processes of the CPU baseline (0 = every core this "
                         "process may use: affinity mask, capped by the cgroup CPU quota)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--save-ppm", default="")
    ap.add_argument("--no-cull", action="store_true", help="force the linear sphere sweep")
    ap.add_argument("--assemble", default="auto", choices=("auto", "host", "gather"),
                    help="N > 1: how the frame reaches host memory. host: every rank's reduce "
                         "writes its interleaved rows into one page-locked shared-memory frame "
                         "(one node); gather: RCCL gather of the rows to rank 0, then a copy to "
                         "host; auto: host when all ranks share a node, else gather")
    ap.add_argument("--gather-fp64", action="store_true",
                    help="N > 1: gather the FP64 accumulators and quantise on rank 0 "
                         "(default: each rank quantises its rows, uint8 gather)")
    ap.add_argument("--no-fixpoint", action="store_true",
                    help="trace provably trapped paths to max_depth (DESIGN.md §9)")
    ap.add_argument("--batch", type=int, default=0,
                    help="frames per trace launch (rt_render_device_frames, <= 32; 0 = auto: "
                         "all timed frames in as few launches as fit, 1 for multi-chunk frames)")
    ap.add_argument("--pipeline", type=int, default=0,
                    help="launches in flight (0 = auto: measured among 1..3 for one-frame "
                         "launches of single-chunk frames, else 1)")
    ap.add_argument("--no-drain-gate", action="store_true",
                    help="frames in flight: start the next launch at once instead of when the "
                         "previous one's work queue empties (rt_context_wait_drain; A/B)")
    ap.add_argument("--no-tail-priority", action="store_true",
                    help="with --pipeline: the draining waves keep their base issue priority "
                         "(RT_FLAG_NO_TAIL_PRIORITY; A/B)")
    ap.add_argument("--chain", action="store_true",
                    help="batched: also try the timed frames as a chain of B/2 or B/4-frame "
                         "launches, two in flight, and keep the fastest (> 1%% gain; r06: C3 "
                         "0.3-0.6%%, shards and C1 / C2 slower, so off by default)")
    ap.add_argument("--no-lean-reduce", action="store_true",
                    help="frames in flight: keep psrt_reduce instead of psrt_reduce_lean (A/B)")
    ap.add_argument("--scaling", default="strong", choices=("weak", "strong"),
                    help="strong (default): the configured frame on any N; weak (study): "
                         "N GPUs render the frame at N x spp (per-GPU work fixed)")
    ap.add_argument("--tune", default="",
                    help="measurement knobs (include/rt.h rt_context_set_tuning), name=value[,...]; "
                         "every knob keeps the output bit-identical")
    ap.add_argument("--emulate-shard", default="",
                    help="R/G: one process renders only rank R's rows of a G-GPU run "
                         "(per-rank step time of the multi-GPU bench, on one GPU; "
                         "no gather, no CPU baseline)")
    return ap.parse_args()


def scene_of(cfg):
    import petershirleyraytracer_amd as P
    if cfg["scene"] == "two":
        return P.scene_two_spheres(), P.camera_default()
    return P.scene_random_spheres(1), P.camera_look_at(aspect=cfg["width"] / cfg["height"])


def host_cpus():
    """The host cores this process may use: the affinity mask, capped by the
    cgroup v2 CPU quota (a GPU box's share of its host); plus nproc and the
    CPU model for the record."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = float(q) / float(period)
    except (OSError, ValueError):
        pass
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    usable = aff if quota is None else max(1, min(aff, int(quota)))
    return dict(nproc=os.cpu_count(), affinity=aff, cgroup_quota=quota, usable=usable,
                cpu_model=model)


def run_reference_rows(O, cfg, args, spp, row0, stride, rows, procs, td, tag="", col_range=None):
    """oracle/_ref/ref_render on `rows` rows (row0, row0 + stride, ...) at `spp`,
    columns (all, or col_range = (c0, c1)) split over `procs` single-thread
    processes. Returns (wall seconds, [(c0, c1, accum[rows, c1 - c0, 3])]) or
    None on failure."""
    w, h = cfg["width"], cfg["height"]
    lo, hi = col_range if col_range else (0, w)
    cols = np.linspace(lo, hi, procs + 1).astype(int)
    cmds = []
    for p in range(procs):
        if cols[p + 1] <= cols[p]:
            continue
        out = os.path.join(td, f"a{tag}{p}.bin")
        cmds.append((cols[p], cols[p + 1], out,
                     [O.REF_BIN, "--scene", cfg["scene"], "--width", str(w), "--height", str(h),
                      "--spp", str(spp), "--depth", str(args.max_depth), "--seed", str(args.seed),
                      "--rows", f"{row0}:{stride}:{rows}", "--cols", f"{cols[p]}:{cols[p + 1]}",
                      "--accum", out]))
    t0 = time.perf_counter()
    running = [subprocess.Popen(c[3], stdout=subprocess.DEVNULL, stderr=subprocess.PIPE)
               for c in cmds]
    ok = all(pr.wait() == 0 for pr in running)
    wall = time.perf_counter() - t0
    if not ok:
        return None
    parts = [(c0, c1, np.fromfile(out, dtype=np.float64).reshape(rows, c1 - c0, 3))
             for c0, c1, out, _ in cmds]
    return wall, parts


def compare_rows(O, parts, frame_acc, row0, stride, rows, spp):
    """Bit-for-bit comparison of reference pixels with the GPU frame's."""
    equal, n_pix, sq = True, 0, 0.0
    sel = frame_acc[row0::stride][:rows]
    for c0, c1, a in parts:
        g = np.ascontiguousarray(sel[:, c0:c1])
        equal &= bool(np.array_equal(a.view(np.uint64), g.view(np.uint64)))
        n_pix += a.shape[0] * a.shape[1]
        d = O.quantize(a, spp).astype(np.float64) - O.quantize(g, spp)
        sq += float(np.sum(d * d))
    mse = sq / max(1, 3 * n_pix)
    psnr = "inf" if mse == 0 else round(10 * math.log10(255.0 ** 2 / mse), 3)
    return dict(pixels_compared=n_pix, fp64_bit_identical=equal, ppm_psnr_db=psnr)


def cpu_baseline(cfg, args, frame_acc):
    """The reference itself (oracle/_ref/ref_render: the reference sources
    compiled unmodified) on a bounded sample of the same workload: a set of
    rows spread over the frame, columns split over one single-thread process
    per usable host core; then one process alone on a smaller set of rows (the
    1-thread rate). Also checks the sampled pixels against the GPU frame bit
    for bit."""
    import oracle as O  # checker / baseline only
    if not O.have_ref():
        return None, None
    w, h, spp = cfg["width"], cfg["height"], cfg["spp"]
    hc = host_cpus()
    procs = args.cpu_procs if args.cpu_procs > 0 else hc["usable"]
    # per-core reference rate: two-sphere 0.62 Ms/s, final 0.0232 Ms/s
    rate = 0.62e6 if cfg["scene"] == "two" else 0.0232e6
    want_samples = args.cpu_seconds * procs * rate
    # rows spread over the whole frame; at most 100 spp per pixel (a sample's
    # cost does not depend on spp, and every pixel's first samples are the same
    # stream prefix), so very high spp still sees the frame's real mix of rays
    spp_eff = min(spp, 100)
    rows = max(1, min(h, int(want_samples / (w * spp_eff))))
    stride = max(1, h // rows)
    rows = len(range(0, h, stride))
    with tempfile.TemporaryDirectory() as td:
        r = run_reference_rows(O, cfg, args, spp_eff, 0, stride, rows, procs, td)
        if r is None:
            return None, None
        wall, parts = r
        samples = rows * w * spp_eff
        parity = compare_rows(O, parts, frame_acc, 0, stride, rows, spp) \
            if frame_acc is not None and spp_eff == spp else None
        # one process alone (1 thread), ~4 s of work: rows spread the same way
        rows1 = max(1, int(4.0 * rate / (w * spp_eff)))
        stride1 = max(1, h // rows1)
        rows1 = len(range(stride1 // 2, h, stride1))
        r1 = run_reference_rows(O, cfg, args, spp_eff, stride1 // 2, stride1, rows1, 1, td, "one")
    one = None if r1 is None else rows1 * w * spp_eff / r1[0] / 1e6
    cb = dict(value=samples / wall / 1e6, unit="Msamples/s", cores=procs, kind="reference",
              one_thread_value=one,
              per_process_value=samples / wall / 1e6 / procs,  # one core's share (1 thread each)
              nproc=hc["nproc"], affinity_cpus=hc["affinity"], cgroup_cpu_quota=hc["cgroup_quota"],
              cpu_model=hc["cpu_model"],
              sample=(f"{rows} rows (every {stride}th) x {w} cols x {spp_eff} spp "
                      f"= {samples} samples of the same workload; reference sources "
                      f"(g++ -O2, unmodified) in {procs} single-thread processes "
                      f"(one per usable core: affinity {hc['affinity']}, cgroup quota "
                      f"{hc['cgroup_quota']}), {wall:.1f} s wall; one_thread_value: "
                      f"{rows1} rows x {w} x {spp_eff} spp in one process"
                      + (f", {r1[0]:.1f} s" if r1 else "")))
    return cb, parity


def reference_parity(cfg, args, frame_acc, world, budget_s=6.0):
    """Sampled pixels of a full frame's FP64 accumulators compared bit for bit
    with the reference itself (oracle/_ref/ref_render) at the frame's full spp:
    whole rows when they fit the budget (~budget_s of CPU on every usable
    core), else a column window of at least `world` rows (C4 at 500 spp, C5 at
    10000). The row stride is odd, so the sampled rows run through every
    residue mod world: every rank's rows are covered."""
    import oracle as O  # checker only
    if not O.have_ref():
        return dict(checked=False, reason="oracle/_ref/ref_render absent")
    w, h, spp = cfg["width"], cfg["height"], cfg["spp"]
    if frame_acc.shape[0] != h:
        return dict(checked=False, reason="weak-scaled frame (not the configured one)")
    procs = host_cpus()["usable"]
    rate = 0.62e6 if cfg["scene"] == "two" else 0.0232e6
    px = max(1, int(budget_s * procs * rate / spp))  # pixels at full spp within the budget
    if px >= world * w:  # whole rows
        rows, cols = max(world, min(h, px // w)), (0, w)
    else:  # a centred column window over max(world, 8) rows
        rows = max(world, min(h, 8))
        nc = max(1, min(w, px // rows))
        c0 = (w - nc) // 2
        cols = (c0, c0 + nc)
    stride = max(1, h // rows) | 1
    rows = len(range(0, h, stride))
    with tempfile.TemporaryDirectory() as td:
        r = run_reference_rows(O, cfg, args, spp, 0, stride, rows, min(procs, cols[1] - cols[0]), td,
                               col_range=cols)
    if r is None:
        return dict(checked=False, reason="reference run failed")
    out = compare_rows(O, r[1], frame_acc, 0, stride, rows, spp)
    out.update(checked=True, rows=f"0::{stride} ({rows} rows)", cols=f"{cols[0]}:{cols[1]}",
               spp=spp, reference_wall_s=round(r[0], 2),
               ranks_covered=len({(k * stride) % world for k in range(rows)}))
    return out


def verify_gathered(cfg, args, frame_acc, world):
    """N > 1: the gathered FP64 frame (a timed frame) against the reference."""
    out = reference_parity(cfg, args, frame_acc, world)
    if out.get("checked"):
        out["gather"] = "RCCL FP64 accumulators" if dist_backend() == "nccl" else dist_backend()
    return out


def dist_backend():
    import torch.distributed as dist
    return dist.get_backend() if dist.is_initialized() else "none"


def profile_counters(config: str):
    """From the committed rocprofv3 PMC summary (profiles/pmc_<config>.json):
    HBM bytes per psrt_trace launch (FETCH_SIZE doubled per the gfx950
    calibration note in MI355X_MICROARCH.md §HBM, + WRITE_SIZE) and the VALU
    issue: SIMD cycles per wave64 VALU instruction, (kernel cycles x 1024
    SIMDs) / SQ_INSTS_VALU, kernel cycles = GRBM_GUI_ACTIVE / 8 XCDs; rocprof's
    VALUBusy, SQ_ACTIVE_INST_VALU x 4 / (kernel cycles x 1024) (quad-cycles
    per wave, so it can pass 1 when 2-cycle instructions overlap); and the
    VALU pipe's busy fraction from the instruction mix, FP64 instructions at
    4 cycles and the others at 2 (SIMD32: a wave64 instruction issues in 2)."""
    path = os.path.join(ROOT, "profiles", f"pmc_{config}.json")
    if not os.path.exists(path):
        return None, None
    try:
        d = json.load(open(path))
        traffic = float(d["hbm_bytes_per_launch"])
    except Exception:
        return None, None
    try:
        c = d["counters"]
        cycles = c["GRBM_GUI_ACTIVE"] / 8
        valu = dict(kernel=d.get("kernel"), insts_per_launch=c["SQ_INSTS_VALU"],
                    salu_insts_per_launch=c.get("SQ_INSTS_SALU"),
                    branch_insts_per_launch=c.get("SQ_INSTS_BRANCH"),
                    kernel_cycles=cycles,
                    simd_cycles_per_valu_inst=round(cycles * 1024 / c["SQ_INSTS_VALU"], 3),
                    note="a wave64 FP64 VALU op holds a SIMD 4 cycles (16 lanes/cycle)",
                    source=f"profiles/pmc_{config}.json")
        simd_cycles = cycles * 1024
        if "SQ_ACTIVE_INST_VALU" in c:
            valu["valu_busy_rocprof"] = round(c["SQ_ACTIVE_INST_VALU"] * 4 / simd_cycles, 4)
        f64 = sum(c.get(k, 0.0) for k in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64",
                                          "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_TRANS_F64"))
        if f64:
            valu["valu_pipe_busy_mix"] = round((4 * f64 + 2 * (c["SQ_INSTS_VALU"] - f64))
                                               / simd_cycles, 4)
        if "SQ_THREAD_CYCLES_VALU" in c and "SQ_ACTIVE_INST_VALU" in c:
            # lanes active per VALU instruction (SIMT divergence), as rocprof's
            # VALUUtilization: SQ_THREAD_CYCLES_VALU / (64 x SQ_ACTIVE_INST_VALU)
            valu["lane_utilisation"] = round(c["SQ_THREAD_CYCLES_VALU"]
                                             / (64.0 * c["SQ_ACTIVE_INST_VALU"]), 4)
    except Exception:
        valu = None
    return traffic, valu


def main():
    args = parse()
    cfg = CONFIGS[args.config]
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and not (world == 1 and args.gpus == 1):
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE",
              file=sys.stderr)

    import torch
    import torch.distributed as dist

    import petershirleyraytracer_amd as P
    from petershirleyraytracer_amd.dist import (HostFrames, gather_frame, gather_frames,
                                                rows_owned, shard)
    from petershirleyraytracer_amd.render import (FLAG_CULL_STATS, FLAG_NO_CULL, FLAG_NO_FIXPOINT,
                                                  FLAG_NO_TAIL_PRIORITY)

    if os.environ.get("PSRT_BENCH_BACKEND", "nccl") != "nccl":
        local = 0  # rehearsal: every rank on the one GPU
    torch.cuda.set_device(local)
    distributed = world > 1 or "TORCHELASTIC_RUN_ID" in os.environ or "MASTER_PORT" in os.environ
    if distributed:  # one process per GPU over RCCL (backend "nccl" on ROCm)
        # PSRT_BENCH_BACKEND=gloo: rehearse N ranks on one GPU (RCCL refuses
        # two ranks on one device); the product path is RCCL
        backend = os.environ.get("PSRT_BENCH_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)

    for kv in filter(None, args.tune.split(",")):  # process defaults: every context takes them
        name, val = kv.split("=")
        P.set_tuning(name.strip(), float(val))
    w, h, spp = cfg["width"], cfg["height"], cfg["spp"]
    spheres, cam = scene_of(cfg)
    config_id = args.config
    # weak scaling: N GPUs (or an emulated shard of G) render N x spp
    n_shards = int(args.emulate_shard.split("/")[1]) if args.emulate_shard else world
    if args.scaling == "weak":
        spp *= n_shards
        if n_shards > 1:
            config_id = f"{args.config}-weak"  # not the configured frame: never read as its number
    # Frames in flight: each slot has its own context (work queue, sample
    # buffer, stats), stream and output rows, so frame k+1 fills the CUs that
    # frame k's last waves release (DESIGN.md §7 "Frame pipelining").
    if args.emulate_shard:
        if world != 1:
            raise SystemExit("--emulate-shard runs in a single process")
        er, eg = (int(x) for x in args.emulate_shard.split("/"))
        off, stride = shard(er, eg)
        rows = rows_owned(h, er, eg)
        args.no_cpu_baseline = True
    else:
        off, stride = shard(rank, world)
        rows = rows_owned(h, rank, world)
    flags = ((FLAG_NO_CULL if args.no_cull else 0)
             | (FLAG_NO_FIXPOINT if args.no_fixpoint else 0))
    prm = P.params(w, h, spp, args.max_depth, args.seed, off, stride, flags)
    prm_notail = P.params(w, h, spp, args.max_depth, args.seed, off, stride,
                          flags | FLAG_NO_TAIL_PRIORITY)
    # the counting kernel variant (sphere / box tests executed), for one untimed frame
    prm_count = P.params(w, h, spp, args.max_depth, args.seed, off, stride,
                         flags | FLAG_CULL_STATS)
    # Frames per launch (--batch; 0 = auto). rt_render_device_frames renders
    # B frames (seeds seed .. seed + B - 1: the same scene and workload, a new
    # sample stream each) in one trace launch, so the launch tail (the last
    # waves' longest paths) is paid once per B frames instead of
    # once per frame. Auto: every timed frame in as few launches as the 32-bit
    # unit ids, the sample buffer and kMaxFrames (32) allow; frames of several
    # sample chunks (C4, C5 on one GPU) go one per launch.
    per_rank = rows * w * spp
    buf_cap = int(P.get_tuning("sample_buf_mb")) << 20  # the library's sample-buffer cap
    multi_chunk = per_rank * SAMPLE_RECORD_BYTES > buf_cap or per_rank >= (1 << 30)
    if args.batch > 0:
        B = min(args.batch, 32)
    elif multi_chunk or per_rank == 0:
        B = 1
    else:
        B = max(1, min(32, args.steps, ((1 << 32) - 1) // per_rank,
                       buf_cap // (per_rank * SAMPLE_RECORD_BYTES)))
    # Frames in flight (one frame per launch only): each slot has its own
    # context (work queue, sample buffer, stats), stream and output rows, so
    # frame k+1 fills the CUs that frame k's last waves release.
    # Two persistent launches that share the GPU for their whole run are slower
    # than one after the other, so batches and multi-chunk frames run one at a
    # time; otherwise the depth is picked by measurement (`tuning` below).
    # Batched: the timed frames in one launch, or (--chain) in launches of
    # B / 2 or B / 4 frames, two in flight: each launch's tail filled by the
    # next and its reduce beside the next trace, only the last exposed
    # (picked by measurement like the one-frame depths; profiles/r06_drain)
    chains = []
    if B > 1 and not multi_chunk and args.chain and args.pipeline == 0:
        chains = sorted({b2 for b2 in ((B + 1) // 2, (B + 3) // 4) if 1 < b2 < B}, reverse=True)
    if args.pipeline > 0:
        candidates = [(args.pipeline, not args.no_tail_priority)]
    elif B > 1 or multi_chunk:
        candidates = [(1, True)]
    else:
        candidates = [(1, True), (2, True), (3, True)]
    depth = max(c[0] for c in candidates)
    # contexts / buffers to allocate: the largest depth tried, and 2 for the
    # one-frame-per-launch comparison beside a batched line (`unbatched`)
    # (one process per GPU only: a rank's extra context is an extra stream
    # and hardware queue, and 8 ranks sharing one GPU in the rehearsal then
    # oversubscribe the queues: C3 8146 -> 7250-7470 Msamples/s, r06_final)
    nslots = max(depth, 2 if B > 1 and not multi_chunk and world == 1 else 1)
    ctxs = []
    scene_ms = []  # rt_context_set_scene: host BVH / grid / neighbour lists + uploads
    for _ in range(nslots):
        c = P.Context(local)
        t0 = time.perf_counter()
        c.set_scene(spheres, cam)
        scene_ms.append((time.perf_counter() - t0) * 1e3)
        ctxs.append(c)
    dev = torch.device("cuda", local)
    # N > 1: how a step's frame reaches host memory (--assemble). "host": the
    # ranks of one node share a page-locked frame (POSIX shared memory) and
    # each rank's psrt_reduce writes its interleaved rows into it across its
    # own GPU's link (rt_context_set_row_pitch): no collective, no copy on
    # rank 0, eight links in parallel instead of rank 0's one. "gather": the
    # RCCL gather over xGMI to rank 0, then rank 0 copies the frame to host.
    assemble = "none"
    if world > 1:
        one_node = int(os.environ.get("LOCAL_WORLD_SIZE", world)) == world
        assemble = args.assemble
        if assemble == "auto":
            assemble = "host" if one_node and not args.gather_fp64 else "gather"
        if assemble == "host" and (not one_node or args.gather_fp64):
            raise SystemExit("--assemble host needs every rank on one node and no --gather-fp64")
    hostframes = None
    assemble_note = None
    if assemble == "host":
        hostframes = HostFrames(nslots * B, h, w, rank, world)
        # every rank must have page-locked the shared frame; otherwise all of
        # them fall back to the gather together (auto) or stop (--assemble host)
        okt = torch.tensor([1 if hostframes.registered else 0], dtype=torch.int32,
                           device=dev if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(okt, op=dist.ReduceOp.MIN)
        if int(okt.item()) == 0:
            why = hostframes.error or "another rank failed"
            hostframes.close()
            hostframes = None
            if args.assemble == "host":
                raise SystemExit(f"--assemble host: rt_host_register failed: {why}")
            assemble, assemble_note = "gather", f"shared host frame unavailable ({why}): gather"
    if assemble == "host":
        for c in ctxs:
            c.set_row_pitch(0, world * w * 3)  # the sums stay packed on the device
    # per slot: B frames' accumulators and bytes
    acc = [torch.zeros((B, rows, w, 3), dtype=torch.float64, device=dev) for _ in range(nslots)]
    rgb = torch.zeros((h, w, 3), dtype=torch.uint8, device=dev) if rank == 0 and world > 1 else None  # --gather-fp64
    rgb_rows = [torch.zeros((B, rows, w, 3), dtype=torch.uint8, device=dev)
                for _ in range(nslots)] if assemble == "gather" else None
    # every step ends with the frame's bytes in pinned host memory (rank 0):
    # per slot and frame, so frames in flight never share one
    host_rows = h if world > 1 else rows
    host_rgb = [torch.empty((B, host_rows, w, 3), dtype=torch.uint8, pin_memory=True)
                for _ in range(nslots)] if rank == 0 and assemble != "host" else None
    # each frame slot renders on its context's own stream
    streams = [torch.cuda.ExternalStream(c.stream(), device=dev) for c in ctxs]
    # N > 1: every gather goes on one stream, in frame order on every rank
    comm = torch.cuda.Stream(dev)

    def barrier():
        if distributed:
            dist.barrier()

    pending = [None] * nslots  # per slot: (timed?, event after the gathers, frames)
    run = {"dn": depth, "kms": [], "rays": [], "exec": [], "frames": [], "prm": prm, "prev": None}

    def ptrs(t, nb):
        # frame f's block by address arithmetic: t[f].data_ptr() builds a view
        # per frame, ~10 us each, paid before the batch's first launch
        base, step = t.data_ptr(), t.stride(0) * t.element_size()
        return [base + f * step for f in range(nb)]

    def launch(i, nb, is_timed):
        """Launch i of a timed() sequence: nb frames in one rt_render_device_frames."""
        sl = i % run["dn"]
        ctx, st = ctxs[sl], streams[sl]
        # frames in flight: this launch starts when the previous one's queue
        # is empty, in its tail (two persistent launches that share the GPU
        # from their start lose more than the tail costs)
        if run["dn"] > 1 and run["prev"] is not None and not args.no_drain_gate:
            ctxs[run["prev"]].wait_drain(st.cuda_stream)
        run["prev"] = sl
        if timeline and is_timed and "tl_call" not in run:
            run["tl_call"] = time.monotonic_ns()
        if world == 1:
            # write_color's bytes go straight into pinned host memory
            # (main.cc:70,86 emit the image): psrt_reduce stores them across
            # the link, so the frame's device-to-host transfer is inside the
            # render and needs no copy of its own (which, as a kernel, would
            # wait for a CU slot behind the next frame's persistent launch)
            ctx.render_device_frames(run["prm"], nb, ptrs(acc[sl], nb), ptrs(host_rgb[sl], nb),
                                     st.cuda_stream)
            pending[sl] = (is_timed, None, nb)
            return
        if hostframes is not None:
            # this rank's rows straight into the shared page-locked frames
            # (slot sl owns frames sl*B .. sl*B + B - 1)
            ctx.render_device_frames(run["prm"], nb, ptrs(acc[sl], nb),
                                     [hostframes.rows_ptr(sl * B + f, w) for f in range(nb)],
                                     st.cuda_stream)
            pending[sl] = (is_timed, None, nb)
            return
        if args.gather_fp64:
            ctx.render_device_frames(run["prm"], nb, ptrs(acc[sl], nb), None, st.cuda_stream)
            src = acc[sl]
        else:
            # write_color is per pixel: each rank quantises its own rows, and
            # the gather moves 3 B per pixel instead of 24 (C3: 2.9 MB, not 23)
            ctx.render_device_frames(run["prm"], nb, ptrs(acc[sl], nb), ptrs(rgb_rows[sl], nb),
                                     st.cuda_stream)
            src = rgb_rows[sl]
        comm.wait_stream(st)
        with torch.cuda.stream(comm):
            # the launch's nb frames in one gather (one collective, one
            # de-interleave per rank), then to pinned host memory on rank 0
            frs = gather_frames(src[:nb], h, rank, world)
            if rank == 0:
                if args.gather_fp64:
                    for f in range(nb):
                        ctxs[sl].quantize_device(frs[f].data_ptr(), w, h, spp, rgb.data_ptr(),
                                                 comm.cuda_stream)
                        host_rgb[sl][f].copy_(rgb, non_blocking=True)
                else:
                    host_rgb[sl][:nb].copy_(frs, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(comm)
        pending[sl] = (is_timed, ev, nb)

    def retire(sl):
        """Wait for the slot's launch (render + gathers) and collect its stats."""
        if pending[sl] is None:
            return
        is_timed, ev, nb = pending[sl]
        st = ctxs[sl].sync_stats()
        if is_timed:
            run["last"] = (sl, nb)  # where the last timed launch's frames are
        if ev is not None:
            ev.synchronize()
        pending[sl] = None
        if is_timed:
            run["kms"].append(st["kernel_ms"])
            run["rays"].append(st["rays"])
            run["frames"].append(nb)
            run["exec"].append((st["tests_executed"], st["box_tests"], st["rays_traced"], nb,
                                st["prerejects"], st["root_box_tests"]))

    def drain():
        for k in range(nslots):
            retire(k)
        torch.cuda.synchronize(dev)

    def batches(n, b):
        out = []
        while n > 0:
            out.append(min(b, n))
            n -= out[-1]
        return out

    timeline = bool(os.environ.get("PSRT_BENCH_TIMELINE"))

    def timed(dn, nwarm, nsteps, b=None, tail=True, count=False):
        """nwarm untimed + nsteps timed frames in launches of up to b frames,
        dn launches in flight; the timed frames start from an idle GPU and end
        when the last one is done."""
        b = b or B
        # launches in flight: each launch's reduce must fit beside the next
        # launch's resident trace, or it waits for that trace's tail
        # (psrt_reduce_lean); the last launch's reduce, with no
        # trace beside it, and one launch at a time: psrt_reduce (faster alone)
        lean = 1 if dn > 1 and not args.no_lean_reduce else 0
        run.update(dn=dn, kms=[], rays=[], exec=[], frames=[], prev=None,
                   prm=prm_count if count else (prm if tail else prm_notail))
        seq = [(nb, False) for nb in batches(nwarm, b)] + [(nb, True) for nb in batches(nsteps, b)]
        t0 = None
        for i, (nb, is_timed) in enumerate(seq):
            if is_timed and t0 is None:
                drain()
                barrier()
                torch.cuda.synchronize(dev)
                t0 = time.perf_counter()
                tl0 = time.monotonic_ns()
            retire(i % dn)  # the slot's previous launch must be done
            ctxs[i % dn].set_tuning("reduce_lean", lean if i < len(seq) - 1 else 0)
            launch(i, nb, is_timed)
        if timeline:
            tl = time.monotonic_ns()
        drain()
        barrier()
        el = time.perf_counter() - t0
        if timeline:  # PSRT_BENCH_TIMELINE: host clock marks to set beside a kernel trace
            print(f"timeline t0_ns={tl0} call_ns={run.pop('tl_call', 0)} enqueued_ns={tl} "
                  f"end_ns={time.monotonic_ns()} "
                  f"boot_minus_mono_ns={time.clock_gettime_ns(time.CLOCK_BOOTTIME) - time.monotonic_ns()}",
                  file=sys.stderr)
        if distributed:
            t = torch.tensor([el], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        return el

    # One-time costs outside the timed steps: set_scene (above) and the
    # camera-ray candidate lists, built by a context's first render and
    # cached (psrt_capi.hip): that render's non-trace device time minus a
    # cached render's
    def one(ctx, sl):
        ctx.render_device_frames(prm, 1, [acc[sl][0].data_ptr()], None, streams[sl].cuda_stream)
        return ctx.sync_stats()
    first = one(ctxs[0], 0)
    again = one(ctxs[0], 0)
    camlist_ms = max(0.0, (first["total_ms"] - first["kernel_ms"])
                     - (again["total_ms"] - again["kernel_ms"]))
    for k in range(1, nslots):
        one(ctxs[k], k)
    # A context's sample buffer grows to its largest render so far: one
    # untimed render of B frames per context here, so no timed launch
    # allocates (with W < B the warmup launch is shorter than a timed one,
    # and the first timed launch would free and re-allocate B frames' records
    # inside the timed region: 0.5-0.8 ms, profiles/r04_timeline)
    if B > 1:
        for k in range(nslots):
            ctxs[k].render_device_frames(prm, B, ptrs(acc[k], B), None, streams[k].cuda_stream)
            ctxs[k].sync_stats()
    torch.cuda.synchronize(dev)

    # untimed tuning runs (one frame per launch only): every candidate depth
    # renders full frames; the fastest (max over ranks) is the one timed below
    tuning = {}
    if len(candidates) > 1:
        for c in candidates:
            nt = max(10, 4 * c[0])
            tuning[str(c[0])] = timed(c[0], 1, nt, 1, c[1]) / nt * 1e3
    # Frames in flight for a gain over 1% in the tuning runs (each launch
    # gated on the previous one's drain, each reduce beside the next trace:
    # rt_context_wait_drain, psrt_reduce_lean)
    depth, tail_prio = candidates[0]
    if tuning:
        best = min(candidates, key=lambda c: tuning[str(c[0])])
        if tuning[str(best[0])] < 0.99 * tuning[str(candidates[0][0])]:
            depth, tail_prio = best
    if chains:
        nt = args.steps
        tuning[f"b{B}x1"] = timed(1, B, nt, B) / nt * 1e3
        for b2 in chains:
            tuning[f"b{b2}x2"] = timed(2, b2, nt, b2) / nt * 1e3
        bb = min(chains, key=lambda b2: tuning[f"b{b2}x2"])
        if tuning[f"b{bb}x2"] < 0.99 * tuning[f"b{B}x1"]:
            B, depth = bb, 2
    elapsed = timed(depth, args.warmup, args.steps, B, tail_prio)
    kernel_ms = sum(run["kms"]) / sum(run["frames"])  # device time of the trace per frame
    rays = sum(run["rays"]) / sum(run["frames"])      # reference rays per frame
    # The timed kernel's own output, kept for the checks after the timed
    # region: the last timed launch's first frame (seed --seed) is the frame
    # compared with the reference (N = 1: the CPU baseline's pixels; N > 1:
    # gathered to rank 0), and its last frame (seed --seed + nb - 1) is
    # compared with a one-frame render of that seed.
    last_sl, last_nb = run["last"]
    timed_first = acc[last_sl][0].clone()
    timed_last = acc[last_sl][last_nb - 1].clone()
    # The same frames one per launch (the unbatched rate, for comparison), and
    # the kernel time for the roofline from one-frame launches one at a time
    # when frames were in flight (their HIP events then span the other frames).
    unbatched = None
    if B > 1:
        # one at a time, then two in flight (gated, the reduce beside the
        # next trace): the faster is the one-frame-per-launch rate
        n1 = min(args.steps, 5)
        el1 = timed(1, 1, n1, 1)
        k1 = round(sum(run["kms"]) / sum(run["frames"]), 3)
        n2 = min(args.steps, 10)
        el2 = timed(2, 2, n2, 1) if nslots >= 2 else float("inf")
        one_ms, two_ms = el1 / n1 * 1e3, el2 / n2 * 1e3
        best_ms = min(one_ms, two_ms)
        unbatched = {"ms_per_step": round(best_ms, 3),
                     "value": round((rows if args.emulate_shard else h) * w * spp / best_ms / 1e3, 4),
                     "frames_in_flight": 2 if two_ms < one_ms else 1,
                     "ms_per_step_one_at_a_time": round(one_ms, 3),
                     "ms_per_step_two_in_flight": round(two_ms, 3) if nslots >= 2 else None,
                     "kernel_ms": k1}
    unpiped = None
    if depth > 1:
        # one launch (of the timed launches' size) at a time: the trace's
        # device time per frame for the roofline, undisturbed by the overlap
        n1 = B if B > 1 else min(args.steps, 3)
        el1 = timed(1, 0, n1, B)
        kernel_ms = sum(run["kms"]) / sum(run["frames"])
        unpiped = {"ms_per_step": round(el1 / n1 * 1e3, 3),
                   "value": round((rows if args.emulate_shard else h) * w * spp * n1 / el1 / 1e6, 4)}
    # Sphere / box tests executed: the timed kernel does not count them (two
    # fewer live registers in its loop), so one untimed frame of the counting
    # variant (RT_FLAG_CULL_STATS, seed `--seed`: frame 0 of every batch)
    # supplies them; the work is deterministic.
    timed(1, 0, 1, 1, count=True)
    executed = run["exec"]
    # the batch check: the timed launch's last frame against a one-frame
    # render of its seed, and its first frame against the counting frame
    # (seed --seed, one frame per launch, the counting kernel variant)
    import hashlib
    torch.cuda.synchronize(dev)
    counted_first = acc[0][0].clone()
    prm_last = P.params(w, h, spp, args.max_depth, args.seed + last_nb - 1, off, stride, flags)
    ctxs[0].render_device_frames(prm_last, 1, [acc[0][0].data_ptr()], None, streams[0].cuda_stream)
    ctxs[0].sync_stats()
    torch.cuda.synchronize(dev)

    def sha(t):
        return hashlib.sha256(t.cpu().numpy().tobytes()).hexdigest()
    batch_check = {
        "frames_in_last_timed_launch": last_nb,
        "last_frame_seed": args.seed + last_nb - 1,
        "last_frame_sha256_timed": sha(timed_last),
        "last_frame_sha256_one_frame_launch": sha(acc[0][0]),
        "first_frame_equal_counting_kernel": bool(torch.equal(timed_first.view(torch.int64),
                                                              counted_first.view(torch.int64))),
    }
    batch_check["last_frame_equal"] = (batch_check["last_frame_sha256_timed"]
                                       == batch_check["last_frame_sha256_one_frame_launch"])
    if world > 1:  # the ranks' checks agree on rank 0 only if all pass
        t = torch.tensor([int(batch_check["last_frame_equal"]
                              and batch_check["first_frame_equal_counting_kernel"])],
                         dtype=torch.int64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        batch_check["all_ranks_equal"] = bool(t.item())
    if world == 1:
        frame = timed_first  # seed --seed, rendered by the timed kernel
        rgb = host_rgb[last_sl][0]

    # an emulated shard processed only its own rows
    total_samples = (rows if args.emulate_shard else h) * w * spp * args.steps
    value = total_samples / elapsed / 1e6

    # per-rank kernel time and HBM fraction (rank 0 reports them all)
    my_kms = float(kernel_ms)
    my_hbm = rows * w * spp * SAMPLE_RECORD_BYTES / (my_kms * 1e-3) / PEAK_HBM if my_kms else 0.0
    per_rank = [dict(rank=0, rows=rows, kernel_ms=round(my_kms, 3), hbm_frac=round(my_hbm, 6))]
    if distributed:
        t = torch.tensor([float(rank), float(rows), my_kms, my_hbm], dtype=torch.float64,
                         device=dev)
        parts = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(parts, t)
        per_rank = [dict(rank=int(p[0]), rows=int(p[1]), kernel_ms=round(float(p[2]), 3),
                         hbm_frac=round(float(p[3]), 6)) for p in (q.cpu() for q in parts)]

    # N > 1 self-check: the timed kernel's frame of seed --seed, its FP64
    # accumulators gathered to rank 0 over the same backend (RCCL), sampled
    # pixels compared bit for bit with the reference itself
    gathered = None
    if world > 1:
        gathered = gather_frame(timed_first, h, rank, world)
        torch.cuda.synchronize(dev)
    host_check = None
    if hostframes is not None and rank == 0:
        # frame 0 of every launch is seed --seed (the untimed launches after
        # the timed region rewrite it with the same bits): the bytes the ranks
        # wrote into host memory against write_color of the gathered FP64 frame
        want = P.quantize(gathered.cpu().numpy(), spp)
        got = hostframes.frames[last_sl * B]
        host_check = {"frames_in_host_memory": nslots * B, "assembled_by": world,
                      "frame_equals_quantized_gathered_fp64": bool(np.array_equal(got, want))}

    if rank == 0:
        n = len(spheres)
        avg_ms = float(kernel_ms)  # psrt_trace device time per frame (launch / frames in it)
        rays_launch = float(rays)  # this rank's reference rays per frame
        tests = rays_launch * n  # sphere::hit calls of the reference algorithm
        nfr = sum(e[3] for e in executed)
        ex_tests = float(np.sum([e[0] for e in executed])) / nfr  # full FP64 sphere tests
        ex_boxes = float(np.sum([e[1] for e in executed])) / nfr  # slab tests evaluated
        ex_rays = float(np.sum([e[2] for e in executed])) / nfr
        ex_pre = float(np.sum([e[4] for e in executed])) / nfr    # FP32 pre-rejects
        ex_root = float(np.sum([e[5] for e in executed])) / nfr   # FP64 root-box tests
        # Algorithmic work of psrt_trace as executed, in FP64-op slots: each
        # kind of test that ran at its operations' measured issue cost
        # (WEIGHTS), plus ~61 FP64 ops per traced ray for the hit record,
        # scatter and RNG trials.
        ex_ops = (ex_tests * WEIGHTS["full_sphere_test"] + ex_pre * WEIGHTS["prereject"]
                  + ex_boxes * WEIGHTS["box_test"] + ex_root * WEIGHTS["root_box_test"]
                  + ex_rays * SHADE_OPS_PER_RAY)
        achieved = ex_ops / (avg_ms * 1e-3)
        ref_equiv = tests * OPS_PER_TEST / (avg_ms * 1e-3)
        # algorithmic HBM bytes of one psrt_trace launch: each sample's record
        # (t: 8 B, k: 2 B) written once; the 485 x 40 B sphere list is L2-resident
        samples_rank = rows * w * spp
        hbm_alg = samples_rank * SAMPLE_RECORD_BYTES
        traffic, valu_issue = profile_counters(args.config)
        out = {
            "metric": METRIC,
            "value": round(value, 4),
            "unit": "Msamples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (procedural scene: final random-spheres, glibc srand(1); counter RNG seed 0)",
            "config": {"workload": cfg["desc"] + (f"; {n_shards} GPUs at {n_shards} x spp (weak scaling: {cfg['spp']} spp of work per GPU)" if args.scaling == "weak" and n_shards > 1 else ""),
                       "config_id": config_id, "width": w, **({"tune": args.tune} if args.tune else {}),
                       "height": h, "spp": spp, "max_depth": args.max_depth, "spheres": n,
                       "parallelism": (f"emulated shard {args.emulate_shard} (rows {off}::{stride})"
                                       if args.emulate_shard else f"interleaved rows x{world}") + ((", RCCL FP64 framebuffer gather" if args.gather_fp64 else ", per-rank write_color into one shared page-locked host frame" if assemble == "host" else ", per-rank write_color + RCCL uint8 gather") if world > 1 else "")},
            "roofline": {
                "bound": "valu",
                "achieved": round(achieved / 1e12, 4),
                "peak": round(PEAK_FP64_OPS / 1e12, 2),
                "unit": "TFLOP/s",
                "frac": round(achieved / PEAK_FP64_OPS, 4),
                "traffic": traffic,
                "kernel": "psrt_trace",
                "avg_launch_ms": round(avg_ms, 3),  # per frame: launch time / frames per launch
                "rays_per_launch": int(rays_launch),
                "rays_traced_per_launch": int(ex_rays),
                "reference_sphere_tests_per_launch": int(tests),
                "full_sphere_tests_per_launch": int(ex_tests),
                "prerejects_per_launch": int(ex_pre),
                "box_tests_evaluated_per_launch": int(ex_boxes),
                "root_box_tests_per_launch": int(ex_root),
                "issue_weights_fp64_slots": {k: round(v, 3) for k, v in WEIGHTS.items()},
                "reference_ops_per_test": OPS_PER_TEST,
                "reference_equivalent_tflops": round(ref_equiv / 1e12, 4),
                "culling": "off (linear sweep)" if (args.no_cull or ex_boxes == 0) else "bvh",
                "shade_ops_per_traced_ray": SHADE_OPS_PER_RAY,
                "fixpoint": not args.no_fixpoint,
                "note": ("VALU-issue bound (FP64 non-FMA op peak 256 CU x 64 lanes x 2.4 GHz); "
                         "achieved = (full FP64 sphere tests, FP32 pre-rejects, FP32 slab tests "
                         "evaluated and FP64 root-box tests, each x its issue_weights_fp64_slots "
                         "(measured instruction costs, scripts/isa_rates.hip), + traced rays x "
                         "61) / avg psrt_trace launch; integer RNG, traversal control and SIMT "
                         "divergence not counted; rays_per_launch = the reference's rays, "
                         "rays_traced = those not proven to end black (DESIGN.md 9); "
                         "reference_equivalent = rays x spheres x 23 / launch; valu_issue: the "
                         "PMC issue rates of the same kernel (profiles/pmc_<config>.json)"),
                "hbm_algorithmic_bytes_per_launch": hbm_alg,
                "hbm_frac": round(hbm_alg / (avg_ms * 1e-3) / PEAK_HBM, 6),
                # measured issue rate (PMC) of the same kernel: the SIMDs' VALU
                # issue is the bound; frac above counts only the FP64 algorithm
                "valu_issue": valu_issue,
            },
            "rays_per_sample": round(float(rays) / (rows * w * spp), 3),
            "frames_per_launch": B,
            # the same frames one per launch (rt_render_device)
            "unbatched": unbatched,
            "frames_in_flight": depth,
            "tail_priority": tail_prio,
            "depth_tuning_ms": {k: round(v, 3) for k, v in tuning.items()} or None,
            # the same frames rendered one at a time (each waits for the last)
            "unpipelined": unpiped,
            "per_rank": per_rank,
            "timed_step": ((f"{B} frames (seeds {args.seed}..{args.seed + B - 1}) per trace launch: " if B > 1 else "")
                           + "render + write_color + " + ("" if assemble in ("none", "host") else "RCCL uint8 gather + " if not args.gather_fp64 else "RCCL FP64 gather + psrt_quantize + ")
                           + ("D2H: every rank's psrt_reduce writes its rows into one shared page-locked host frame" if assemble == "host" else
                              "D2H of the frame's bytes into pinned host memory (rank 0)" if world > 1 else
                              "D2H: psrt_reduce writes the frame's bytes into pinned host memory")),
            "frame_to_host": assemble if assemble_note is None else assemble_note,
            # one-time costs, outside the timed steps
            "one_time_ms": {"set_scene": round(scene_ms[0], 3),
                            "camera_lists": round(camlist_ms, 3),
                            "note": "set_scene: host BVH / grid / neighbour lists + uploads "
                                    "(wall); camera_lists: psrt_camera_lists, first render's "
                                    "non-trace device time minus a cached render's"},
        }
        if args.save_ppm and rgb is not None:
            P.write_ppm(args.save_ppm, rgb.cpu().numpy(), binary=True)
        out["batch_check"] = batch_check
        if host_check is not None:
            out["host_frame_check"] = host_check
        cb, parity = None, None
        if world == 1 and not args.no_cpu_baseline:
            try:
                cb, parity = cpu_baseline(cfg, args, frame.cpu().numpy())
            except Exception as e:  # baseline is reported, never the target
                print(f"cpu baseline failed: {e}", file=sys.stderr)
            if parity is None and not args.emulate_shard:
                # spp > 100 (C4, C5): the baseline's rate sample runs at 100 spp,
                # so the timed frame is checked at its full spp on a column window
                try:
                    parity = reference_parity(cfg, args, frame.cpu().numpy(), 1)
                except Exception as e:  # reported, never the target
                    parity = dict(checked=False, reason=f"{type(e).__name__}: {e}")
        if world > 1:
            try:
                parity = verify_gathered(cfg, args, gathered.cpu().numpy(), world)
            except Exception as e:  # reported, never the target
                parity = dict(checked=False, reason=f"{type(e).__name__}: {e}")
        out["cpu_baseline"] = cb
        out["parity_vs_cpu"] = parity
        print(json.dumps(out), flush=True)

    # Teardown order matters: torch's pinned-host allocator keeps an event on
    # each stream a copy into host_rgb ran on (the contexts' own streams), so
    # those buffers go before close() destroys the streams.
    torch.cuda.synchronize(dev)
    host_rgb = None
    streams.clear()
    import gc
    gc.collect()
    torch.cuda.synchronize(dev)
    for c in ctxs:
        c.close()
    if hostframes is not None:
        hostframes.close()
    if distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
