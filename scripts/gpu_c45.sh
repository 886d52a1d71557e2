#!/bin/bash
# GPU parity suite, then C4 and C5 on one GPU with the default sample buffer.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config c4 --steps 3 --warmup 1 --cpu-seconds 8 > gpurun_out/bench_c4.log 2>&1
rc=$?; echo "c4 rc=$rc"; tail -1 gpurun_out/bench_c4.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config c5 --steps 2 --warmup 1 --cpu-seconds 8 > gpurun_out/bench_c5.log 2>&1
rc=$?; echo "c5 rc=$rc"; tail -1 gpurun_out/bench_c5.log | cut -c1-400; exit $rc
