#!/bin/bash
# per-kernel durations of a bench run: KT_ARGS="--emulate-shard 0/64" bash scripts/gpu_ktrace.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/ktrace
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 bench.py --no-cpu-baseline --steps ${STEPS:-3} --warmup 1 ${KT_ARGS} > $OUT/run.log 2>&1 || exit $?
python3 - <<'PY'
import csv, glob
for f in glob.glob("gpurun_out/ktrace/**/run_kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print(f"{r['Name'][:90]:90s} calls={r['Calls']:>4s} avg_us={float(r['AverageNs'])/1e3:9.1f}")
PY
