#!/bin/bash
# parity subset, then an env-knob sweep of the bench (kernel time only).
# SWEEP="PSRT_RNG_FILL=1 PSRT_BATCH=24,PSRT_REFILL_MIN=16 ..." (each item: comma-joined env settings)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_gpu_culling.py tests/test_gpu_parity.py -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
i=0
for kv in ${SWEEP:-DEFAULT=1}; do
  i=$((i+1))
  env ${kv//,/ } timeout -k 10 300 python bench.py --no-cpu-baseline --steps ${STEPS:-10} ${BENCH_ARGS} > gpurun_out/sweep_$i.log 2>&1
  rc=$?; [ $rc -eq 0 ] || exit $rc
  python3 -c "import json; d=json.loads(open('gpurun_out/sweep_$i.log').read().strip().splitlines()[-1]); print('$kv', d['value'], d['roofline']['avg_launch_ms'])"
done
env ${STAMP_ENV:-DEFAULT=1} PSRT_STAMPS=1 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 1 ${BENCH_ARGS} > gpurun_out/bench_stamps.log 2>&1
grep -E "psrt_sections|psrt_util" gpurun_out/bench_stamps.log | tail -2
