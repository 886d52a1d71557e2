#!/bin/bash
# parity subset + bench + section-stamp diagnostic (shares only)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_gpu_culling.py tests/test_gpu_parity.py -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 600 python bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log | cut -c1-900; [ $rc -eq 0 ] || exit $rc
PSRT_STAMPS=1 timeout -k 10 600 python bench.py --no-cpu-baseline --steps 1 ${BENCH_ARGS} > gpurun_out/bench_stamps.log 2>&1
rc=$?; echo "stamps rc=$rc"; grep psrt_sections gpurun_out/bench_stamps.log | tail -1
exit $rc
