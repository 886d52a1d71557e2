"""Summarise a rocprofv3 session (scripts/gpu_profile.sh output) into profiles/.

    python scripts/summarize_profile.py gpurun_out/prof_c3 profiles/r01 c3 [N_UNPIPELINED]

Writes <dst>/kernel_stats_<cfg>.csv (the --stats summary as produced),
<dst>/pmc_<cfg>.csv (per-dispatch counters of the psrt kernels) and
profiles/pmc_<cfg>.json (per-launch HBM bytes + derived rates that bench.py
reads for roofline.traffic). Only the timed kernel variant (TIMED below)
enters the summary: counters, kernel_stats and dispatch durations alike. gfx950 corrections (MI355X_MICROARCH.md §HBM):
FETCH_SIZE counts half the bytes of wide coalesced reads -> doubled; counters
are in KiB; GRBM_GUI_ACTIVE sums the 8 XCDs.
"""
import csv
import glob
import json
import os
import shutil
import sys

src, dst, cfg = sys.argv[1], sys.argv[2], sys.argv[3]
os.makedirs(dst, exist_ok=True)
stats = os.path.join(src, "trace", "run_kernel_stats.csv")
shutil.copy(stats, os.path.join(dst, f"kernel_stats_{cfg}.csv"))
# The timed kernel of bench.py is the default (non-counting) variant
# psrt_trace<kBVH, kStamps, kLds, kCount> = <true, false, true, false>; the
# bench also runs one untimed RT_FLAG_CULL_STATS frame (<..., true>), whose
# counters, duration and kernel_stats row must not stand for the timed one.
TIMED = os.environ.get("PSRT_TIMED_KERNEL", "psrt_trace<true, false, true, false>")


def is_timed(name):
    return TIMED in name


rows = []
for f in sorted(glob.glob(os.path.join(src, "pmc_*", "run_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        if "psrt" in r["Kernel_Name"]:
            rows.append(r)
with open(os.path.join(dst, f"pmc_{cfg}.csv"), "w", newline="") as f:
    keys = ["Kernel_Name", "Counter_Name", "Counter_Value", "Grid_Size", "Workgroup_Size",
            "VGPR_Count", "SGPR_Count", "LDS_Block_Size", "Start_Timestamp", "End_Timestamp"]
    w = csv.DictWriter(f, fieldnames=keys)
    w.writeheader()
    for r in rows:
        w.writerow({k: r[k] for k in keys})
# per counter: the mean over the timed kernel's dispatches (one per PMC pass
# and timed frame; the counting frame's dispatches are left out)
vals = {}
for r in rows:
    if is_timed(r["Kernel_Name"]):
        vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
c = {k: sum(v) / len(v) for k, v in vals.items()}
dispatches = {k: len(v) for k, v in vals.items()}
avg = {}
for line in csv.DictReader(open(stats)):
    if is_timed(line["Name"]):
        avg = dict(kernel=line["Name"][:80], calls=int(line["Calls"]),
                   average_ns=float(line["AverageNs"]))
# per-dispatch durations: the first launch is bench.py's warmup step, which
# bench.py's own HIP-event average leaves out; report the timed launches too
trace = os.path.join(src, "trace", "run_kernel_trace.csv")
if os.path.exists(trace):
    d = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
         for r in csv.DictReader(open(trace)) if is_timed(r["Kernel_Name"])]
    if len(d) > 1:
        avg["average_ns_after_warmup"] = sum(d[1:]) / len(d[1:])
    # bench.py renders its timed frames pipelined (a dispatch's span then
    # includes the neighbouring frame's work), then min(steps, 3) frames one
    # at a time; its roofline kernel time is the average of those last ones
    n1 = int(sys.argv[4]) if len(sys.argv) > 4 else 0
    if n1 and len(d) > n1:
        avg["average_ns_unpipelined"] = sum(d[-n1:]) / n1
    # multi-frame launches (bench.py batches its timed frames, B per launch):
    # the batched dispatches are the long ones; their duration per frame is
    # what bench.py's roofline divides by (PSRT_FRAMES_PER_LAUNCH=B)
    fpl = int(os.environ.get("PSRT_FRAMES_PER_LAUNCH", "1"))
    if fpl > 1 and d:
        long_ = [x for x in d if x >= 0.5 * max(d)]
        avg["frames_per_launch"] = fpl
        avg["batched_dispatches"] = len(long_)
        avg["average_ns_per_frame_batched"] = sum(long_) / len(long_) / fpl
    avg["dispatch_ns"] = d
fetch = c.get("FETCH_SIZE", 0.0) * 1024 * 2
write = c.get("WRITE_SIZE", 0.0) * 1024
# The counters are per PMC dispatch (one-frame launches: the PMC passes run
# bench.py --steps 1), so rates divide by those dispatches' own durations
# (Start/End_Timestamp of the counter rows, ns), not by the kernel-trace
# run's average, whose multi-frame dispatches are 20x longer.
pmc_ns = {}
for r in rows:
    if is_timed(r["Kernel_Name"]):
        a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        pmc_ns[(r["Counter_Name"], a, b)] = b - a
durs = {}
for (name, _, _), ns in pmc_ns.items():
    durs.setdefault(name, []).append(ns)
pmc_secs = {k: sum(v) / len(v) * 1e-9 for k, v in durs.items()}
t_all = [ns for v in durs.values() for ns in v]
secs = sum(t_all) / len(t_all) * 1e-9 if t_all else 0.0
t_fetch, t_write = pmc_secs.get("FETCH_SIZE", secs), pmc_secs.get("WRITE_SIZE", secs)
t_grbm = pmc_secs.get("GRBM_GUI_ACTIVE", secs)
out = {
    "kernel": TIMED, "config": cfg, "kernel_stats": avg, "pmc_dispatches": dispatches,
    "pmc_dispatch_ms": round(secs * 1e3, 4),
    "hbm_bytes_per_launch": fetch + write,
    "fetch_bytes_per_launch_x2": fetch, "write_bytes_per_launch": write,
    "hbm_gbps": (fetch / t_fetch + write / t_write) / 1e9 if t_fetch and t_write else None,
    "clock_ghz": c["GRBM_GUI_ACTIVE"] / 8 / t_grbm / 1e9 if t_grbm and "GRBM_GUI_ACTIVE" in c else None,
    "rate_note": "hbm_gbps / clock_ghz: per PMC dispatch, over that pass's own dispatch durations",
    "counters": c,
}
if "SQ_INSTS_VALU" in c and "SQ_WAVES" in c:
    out["valu_insts_per_wave"] = c["SQ_INSTS_VALU"] / c["SQ_WAVES"]
if "SQ_WAIT_INST_ANY" in c and c.get("SQ_WAVE_CYCLES"):
    # wave cycles spent waiting for an instruction's operands (latency)
    out["wait_inst_frac"] = c["SQ_WAIT_INST_ANY"] / c["SQ_WAVE_CYCLES"]
if "GRBM_GUI_ACTIVE" in c:
    cyc = c["GRBM_GUI_ACTIVE"] / 8  # one XCD's clock over the launch
    for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_BRANCH"):
        if k in c and c[k]:
            out[f"simd_cycles_per_{k[9:].lower()}"] = cyc * 1024 / c[k]
json.dump(out, open(os.path.join(ROOT := os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                 "profiles", f"pmc_{cfg}.json"), "w"), indent=1)
json.dump(out, open(os.path.join(dst, f"pmc_{cfg}.json"), "w"), indent=1)
print(json.dumps({k: v for k, v in out.items() if k != "counters"}, indent=1))
