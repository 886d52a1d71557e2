#!/bin/bash
# VALU/SALU instruction counts of psrt_trace per variant (deterministic-ish,
# unlike timings): VARIANTS="DEFAULT=1 PSRT_LIB=...,PSRT_X=1" bash scripts/gpu_insts.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
for kv in ${VARIANTS:-DEFAULT=1}; do
  i=$((i+1))
  d=gpurun_out/insts_$i
  env ${kv//,/ } timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES --output-format csv -d $d -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline ${BENCH_ARGS} > $d.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "$kv rc=$rc"; tail -5 $d.log; exit $rc; }
  python3 - "$kv" "$d" <<'PY'
import csv, glob, sys
kv, d = sys.argv[1], sys.argv[2]
tot = {}
for f in glob.glob(d + "/**/run_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "psrt_trace" in r["Kernel_Name"]:
            tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
print(kv, {k: f"{v/1e9:.3f}G" for k, v in sorted(tot.items())})
PY
done
