#!/bin/bash
# Bench one config under several environment settings (runtime knobs), ROUNDS
# times interleaved: ENVS="A=1,B=2 C=3 ..." (comma-separated assignments per
# variant; "-" = no extra setting). LIB selects a library build (default libpsrt.so).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/env
CFG=${CONFIG:-c3}
L=${LIB:-petershirleyraytracer_amd/lib/libpsrt.so}
for r in $(seq 1 ${ROUNDS:-1}); do
  for v in ${ENVS:--}; do
    tag=$(echo "$v" | tr ',=' '_-')
    if [ "$v" = "-" ]; then set --; else set -- $(echo "$v" | tr ',' ' '); fi
    env PSRT_LIB=$L "$@" timeout -k 10 120 python bench.py --config $CFG --no-cpu-baseline --steps ${STEPS:-10} --warmup 2 ${BENCH_ARGS} > gpurun_out/env/b_${tag}_$r.log 2>&1 || { echo "bench $v failed"; tail -5 gpurun_out/env/b_${tag}_$r.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/env/b_${tag}_$r.log').read().strip().splitlines()[-1]); print('$v round $r', 'ms/step', d['ms_per_step'], 'kernel ms', d['roofline']['avg_launch_ms'], 'Msamples/s', d['value'])"
  done
done
