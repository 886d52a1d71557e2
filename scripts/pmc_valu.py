"""Mean per-dispatch PMC counters of the timed psrt_trace kernel from a
rocprofv3 --pmc output directory (run_counter_collection.csv), one JSON line.

    python scripts/pmc_valu.py <dir> [kernel-substring]
"""
import csv
import glob
import json
import os
import sys

d = sys.argv[1]
want = sys.argv[2] if len(sys.argv) > 2 else "psrt_trace<true, false, true, false>"
vals, durs = {}, {}
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if want in r["Kernel_Name"]:
            vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
            durs[(r["Start_Timestamp"], r["End_Timestamp"])] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
out = {k: sum(v) / len(v) for k, v in vals.items()}
out["dispatch_ms"] = sum(durs.values()) / max(1, len(durs)) * 1e-6
out["dispatches"] = len(durs)
print(json.dumps(out))
