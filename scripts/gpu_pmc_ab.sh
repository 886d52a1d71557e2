#!/bin/bash
# One PMC pass per environment variant (ENVS as in gpu_envs.sh) on one frame
# of CONFIG: psrt_trace counters per launch.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcab
CFG=${CONFIG:-c3}
CTRS=${CTRS:-"SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES"}
for v in ${ENVS:--}; do
  tag=$(echo "$v" | tr ',=' '_-')
  if [ "$v" = "-" ]; then set --; else set -- $(echo "$v" | tr ',' ' '); fi
  rm -rf gpurun_out/pmcab/$tag
  env "$@" timeout -s KILL 120 rocprofv3 --pmc $CTRS --output-format csv -d gpurun_out/pmcab/$tag -o run -- python3 bench.py --config $CFG --steps 1 --warmup 0 --pipeline 1 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/pmcab/$tag.log 2>&1 || { echo "pmc $v failed"; tail -3 gpurun_out/pmcab/$tag.log; exit 1; }
  python3 - "$tag" <<'PY'
import csv, glob, sys, collections
v = sys.argv[1]
c = collections.defaultdict(float); n = collections.Counter()
for f in glob.glob(f"gpurun_out/pmcab/{v}/**/run_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "psrt_trace" in r["Kernel_Name"]:
            c[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
k = max(n.values()) if n else 1
print(v, "per launch (M):", {x: round(y / k / 1e6, 2) for x, y in sorted(c.items())}, "launches", k)
PY
done
