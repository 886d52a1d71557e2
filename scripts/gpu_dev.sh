#!/bin/bash
# development loop: chosen GPU tests, then the default bench (no CPU baseline)
# and the diagnostic section stamps. TESTS="tests/x.py::y ..." (default: all gpu)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 ${PYTEST_TIMEOUT:-600} python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_dev.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_dev.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/bench_dev.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_dev.log | cut -c1-600; [ $rc -eq 0 ] || exit $rc
if [ -n "$STAMPS" ]; then
PSRT_STAMPS=1 timeout -k 10 120 python bench.py --no-cpu-baseline --steps 1 --warmup 1 --pipeline 1 ${BENCH_ARGS} > gpurun_out/stamps_dev.log 2>&1
rc=$?; echo "stamps rc=$rc"; grep -E "psrt_sections|psrt_util" gpurun_out/stamps_dev.log | tail -2
fi
exit $rc
