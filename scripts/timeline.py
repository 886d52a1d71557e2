"""Sets bench.py's PSRT_BENCH_TIMELINE host marks beside a rocprofv3 kernel
trace of the same run: per timed region, the host's enqueue time, the gap to
the first kernel, the kernels and the end of the sync (ms from t0).

  python3 scripts/timeline.py <kernel_trace.csv> <bench stderr>
"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
for line in open(sys.argv[2]):
    if not line.startswith("timeline"):
        continue
    t = {k: int(v) for k, v in re.findall(r"(\w+)=(-?\d+)", line)}
    t0, t1 = t["t0_ns"], t["end_ns"]
    print(f"region {(t1 - t0) / 1e6:.3f} ms: call at {(t['call_ns'] - t0) / 1e6:.3f}, "
          f"enqueued at {(t['enqueued_ns'] - t0) / 1e6:.3f}")
    for s, e, n in ks:
        if t0 <= s <= t1:
            print(f"  {(s - t0) / 1e6:9.3f} +{(e - s) / 1e6:8.3f}  {n[:50]}")
