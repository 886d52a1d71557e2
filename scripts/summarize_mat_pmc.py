"""Summarise the material kernel's PMC passes (scripts/gpu_mat_pmc.sh) into
profiles/pmc_mat.json: counters averaged over the psrt_trace_mat dispatches of
the timed (non-counting) variant, kernel cycles (GRBM_GUI_ACTIVE / 8 XCDs) and
SIMD cycles per VALU instruction. scripts/bench_materials.py reads it.

    python scripts/summarize_mat_pmc.py gpurun_out/prof_mat_pmc
"""
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = sys.argv[1]
vals = collections.defaultdict(list)
for f in sorted(glob.glob(os.path.join(src, "pmc_*", "run_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        if "psrt_trace_mat<" not in name:
            continue
        targs = name.split("psrt_trace_mat<", 1)[1].split(">", 1)[0].split(",")
        if targs[-1].strip() == "false":  # kCount = false: the timed variant
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
c = {k: sum(v) / len(v) for k, v in vals.items()}
out = {"kernel": "psrt_trace_mat (timed variant)", "counters": c,
       "pmc_dispatches": {k: len(v) for k, v in vals.items()}}
if "GRBM_GUI_ACTIVE" in c and "SQ_INSTS_VALU" in c:
    cyc = c["GRBM_GUI_ACTIVE"] / 8
    out["kernel_cycles"] = cyc
    out["simd_cycles_per_valu"] = cyc * 1024 / c["SQ_INSTS_VALU"]
if "SQ_WAIT_INST_ANY" in c and "SQ_WAVE_CYCLES" in c:
    out["wait_inst_frac"] = c["SQ_WAIT_INST_ANY"] / c["SQ_WAVE_CYCLES"]
json.dump(out, open(os.path.join(ROOT, "profiles", "pmc_mat.json"), "w"), indent=1)
print(json.dumps({k: v for k, v in out.items() if k != "counters"}, indent=1))
