#!/bin/bash
# r03: the new bench tests (N=1 line, N=2 gloo rehearsal with gathered parity),
# then a PC-sampling attempt of psrt_trace.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_bench.py tests/test_gpu_culling_kat.py -x -v --timeout 150 --timeout-method thread > gpurun_out/pytest_bench.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_bench.log
[ $rc -le 1 ] || exit $rc
INTERVAL=${INTERVAL:-65536} bash scripts/gpu_pcsample.sh
