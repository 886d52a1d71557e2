#!/bin/bash
# r04 final (second, after the walk-tail and bench-sizing changes): the whole GPU suite, smoke, the driver's default bench line,
# a 20-step C3 bench, and C1 / C2 / C4 / C5 bench lines.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r04_final2
O=gpurun_out/r04_final2
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > $O/bench_default.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench_c3.log 2>&1 || exit $?
for c in c1 c2; do timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_$c.log 2>&1 || exit $?; done
for c in c4 c5; do timeout -k 10 300 python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_$c.log 2>&1 || exit $?; done
for f in $O/bench_*.log; do python3 -c "import json,sys; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); print('$f', round(d['value'],1), d['ms_per_step'], d['roofline']['avg_launch_ms'] if d.get('roofline') else None, d.get('frames_per_launch'))"; done
