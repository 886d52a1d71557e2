#!/bin/bash
# A/B of library builds: for each lib in $LIBS (names under
# petershirleyraytracer_amd/lib/libpsrt_<name>.so, or "cur" = libpsrt.so):
# bench ms/step + kernel ms (C3 by default), then one PMC pass counting the
# trace kernel's VALU / SALU instructions. ROUNDS repeats the bench list
# (interleaved, to average out clock drift).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/var
CFG=${CONFIG:-c3}
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in ${LIBS:-cur}; do
    L=petershirleyraytracer_amd/lib/libpsrt_$v.so; [ "$v" = cur ] && L=petershirleyraytracer_amd/lib/libpsrt.so
    PSRT_LIB=$L timeout -k 10 120 python bench.py --config $CFG --no-cpu-baseline --steps ${STEPS:-10} --warmup 2 ${BENCH_ARGS} > gpurun_out/var/b_${v}_$r.log 2>&1 || { echo "bench $v failed"; tail -5 gpurun_out/var/b_${v}_$r.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/var/b_${v}_$r.log').read().strip().splitlines()[-1]); print('$v round $r', 'ms/step', d['ms_per_step'], 'unpiped', d.get('unpipelined',{}).get('ms_per_step'), 'kernel ms', d['roofline']['avg_launch_ms'], 'Msamples/s', d['value'])"
  done
done
if [ -n "$PMC" ]; then
for v in ${LIBS:-cur}; do
  L=petershirleyraytracer_amd/lib/libpsrt_$v.so; [ "$v" = cur ] && L=petershirleyraytracer_amd/lib/libpsrt.so
  rm -rf gpurun_out/var/pmc_$v
  PSRT_LIB=$L timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_BRANCH --output-format csv -d gpurun_out/var/pmc_$v -o run -- python3 bench.py --config $CFG --steps 1 --warmup 0 --pipeline 1 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/var/pmc_$v.log 2>&1 || { echo "pmc $v failed"; exit 1; }
  python3 - "$v" <<'PY'
import csv, glob, sys, collections
v = sys.argv[1]
c = collections.defaultdict(float)
n = collections.Counter()
for f in glob.glob(f"gpurun_out/var/pmc_{v}/**/run_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "psrt_trace" in r["Kernel_Name"]:
            c[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
k = max(n.values()) if n else 1
print(v, "per launch:", {x: round(y / k / 1e6, 2) for x, y in sorted(c.items())}, "(M; launches", k, ")")
PY
done
fi
