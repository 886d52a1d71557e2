#!/bin/bash
# parity subset, then PSRT_BATCH sweep of the bench (kernel time only)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_gpu_culling.py tests/test_gpu_parity.py -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
for b in ${BATCHES:-1 8 16 24 32 48}; do
  PSRT_BATCH=$b timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 > gpurun_out/bench_b$b.log 2>&1
  rc=$?; [ $rc -eq 0 ] || exit $rc
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/bench_b$b.log').read().strip().splitlines()[-1]); print('batch $b', d['value'], d['roofline']['avg_launch_ms'])"
done
PSRT_STAMPS=1 PSRT_BATCH=${STAMP_BATCH:-24} timeout -k 10 300 python bench.py --no-cpu-baseline --steps 1 > gpurun_out/bench_stamps.log 2>&1
grep psrt_sections gpurun_out/bench_stamps.log | tail -1
