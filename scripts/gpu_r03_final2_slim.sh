#!/bin/bash
# r03 final (slim): GPU suite, smoke, the driver's default bench line and a
# 20-step C3 line, then the rocprofv3 trace + PMC passes of C3 (gpu_profile.sh)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r03_final2
O=gpurun_out/r03_final2
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > $O/bench_default.log 2>&1 || exit $?
tail -1 $O/bench_default.log | cut -c1-200
CONFIG=c3 STEPS=20 bash scripts/gpu_profile.sh || exit $?
for c in c2 c4; do timeout -k 10 300 python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_$c.log 2>&1 || exit $?; done
