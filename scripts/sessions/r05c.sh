#!/bin/bash
# r05 session C: the GPU suite and smoke after the escape table's removal, the
# bench lines (default with the CPU baseline; C1, C2, C4, C5) and the material
# bench (frames batched per launch, and one per launch).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05c
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > $O/bench_default.log 2>&1 || exit $?
for c in c1 c2 c4 c5; do
  timeout -k 10 400 python bench.py --config $c --no-cpu-baseline > $O/bench_$c.log 2>&1 || exit $?
  echo "bench $c done"
done
timeout -k 10 300 python scripts/bench_materials.py > $O/mat_batched.log 2>&1 || exit $?
timeout -k 10 300 python scripts/bench_materials.py --batch 1 --cpu-rows 1 > $O/mat_one.log 2>&1 || exit $?
for f in $O/bench_*.log $O/mat_*.log; do python3 -c "import json; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); r=d['roofline']; print('$f', round(d['value'],1), d['ms_per_step'], r['avg_launch_ms'], r['frac'])"; done
