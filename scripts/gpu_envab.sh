#!/bin/bash
# A/B of runtime knobs: for each "NAME=ENV1,ENV2" in $VARIANTS (ENV "-" = none):
# bench ms/step + kernel ms, and (PMC=1) one PMC pass of VALU / SALU / cycles.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/envab
CFG=${CONFIG:-c3}
for r in $(seq 1 ${ROUNDS:-2}); do
  for spec in ${VARIANTS}; do
    name=${spec%%=*}; envs=${spec#*=}; envs=${envs//,/ }; [ "$envs" = "-" ] && envs=""
    env $envs timeout -k 10 120 python bench.py --config $CFG --no-cpu-baseline --steps ${STEPS:-10} --warmup 2 ${BENCH_ARGS} > gpurun_out/envab/b_${name}_$r.log 2>&1 || { echo "bench $name failed"; tail -5 gpurun_out/envab/b_${name}_$r.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/envab/b_${name}_$r.log').read().strip().splitlines()[-1]); print('$name round $r', 'ms/step', d['ms_per_step'], 'kernel ms', d['roofline']['avg_launch_ms'], 'Msamples/s', d['value'])"
  done
done
if [ -n "$PMC" ]; then
for spec in ${VARIANTS}; do
  name=${spec%%=*}; envs=${spec#*=}; envs=${envs//,/ }; [ "$envs" = "-" ] && envs=""
  rm -rf gpurun_out/envab/pmc_$name
  for e in $envs; do export "$e"; done
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE SQ_INSTS_VMEM SQ_INSTS_BRANCH --output-format csv -d gpurun_out/envab/pmc_$name -o run -- python3 bench.py --config $CFG --steps 1 --warmup 0 --pipeline 1 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/envab/pmc_$name.log 2>&1 || { echo "pmc $name failed"; exit 1; }
  for e in $envs; do unset "${e%%=*}"; done
  python3 - "$name" <<'PY'
import csv, glob, sys, collections
v = sys.argv[1]
c = collections.defaultdict(float)
n = collections.Counter()
for f in glob.glob(f"gpurun_out/envab/pmc_{v}/**/run_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "psrt_trace" in r["Kernel_Name"]:
            c[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
k = max(n.values()) if n else 1
print(v, "per launch:", {x: round(y / k / 1e6, 2) for x, y in sorted(c.items())}, "(M; launches", k, ")")
PY
done
fi
