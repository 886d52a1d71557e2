#!/bin/bash
# r05 session B: the GPU suite (device groups, far camera, material fault hook,
# overlapping frame buffers, escape table), smoke, the default bench line and
# the escape-table A/B (--tune no_escape=1), then the C3 rocprofv3 trace + PMC passes.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05b
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > $O/bench_default.log 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --tune no_escape=1 > $O/bench_noesc_$i.log 2>&1 || exit $?
  timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_esc_$i.log 2>&1 || exit $?
done
for f in $O/bench_*.log; do python3 -c "import json; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); r=d['roofline']; print('$f', round(d['value'],1), d['ms_per_step'], r['avg_launch_ms'], r['frac'], r['box_tests_evaluated_per_launch'], r['rays_traced_per_launch'])"; done
OUTDIR=$O/prof_c3 CONFIG=c3 STEPS=2 bash scripts/gpu_profile.sh || exit $?
