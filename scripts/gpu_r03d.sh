#!/bin/bash
# r03: multi-frame launches: the context tests, then bench C3 (auto batch) and C1/C2.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_context.py tests/test_gpu_bench.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_ctx.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_ctx.log
[ $rc -le 1 ] || exit $rc
for c in c3 c2 c1; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_$c.log 2>&1
  rc=$?; echo "bench $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
