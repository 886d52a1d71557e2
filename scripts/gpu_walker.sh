#!/bin/bash
# Walk server A/B: GPU parity suite, then C3 with and without the walker.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
for v in "" "PSRT_NO_WALKER=1" ${EXTRA_VARIANTS}; do
  tag=${v:-walker}
  env $v timeout -k 10 240 python bench.py --steps 10 --warmup 2 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/bench_$tag.log 2>&1
  rc=$?; echo "bench $tag rc=$rc"
  python - gpurun_out/bench_$tag.log <<'PY'
import json,sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d=json.loads(l); r=d['roofline']
        print(f"  value {d['value']:.1f} ms/step {d['ms_per_step']} kernel {r['avg_launch_ms']} unpiped {d['unpipelined']} boxes {r['executed_box_tests_per_launch']} tests {r['executed_sphere_tests_per_launch']}")
PY
  [ $rc -eq 0 ] || exit $rc
done
