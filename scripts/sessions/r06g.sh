#!/bin/bash
# r06 session G: the final tree's records: GPU suite, smoke, the default bench
# line (the driver's command) and two more C3 lines, one frame per launch, C1,
# C2, C4, C5, the material bench (batched and one frame per launch).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06g
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > $O/bench_default.log 2>&1 || exit $?
for i in 2 3; do timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_c3_$i.log 2>&1 || exit $?; done
timeout -k 10 300 python bench.py --no-cpu-baseline --batch 1 > $O/bench_c3_batch1.log 2>&1 || exit $?
for c in c1 c2; do timeout -k 10 300 python bench.py --config $c --cpu-seconds 3 > $O/bench_$c.log 2>&1 || exit $?; done
for c in c4 c5; do timeout -k 10 600 python bench.py --config $c --cpu-seconds 3 > $O/bench_$c.log 2>&1 || exit $?; done
timeout -k 10 300 python scripts/bench_materials.py > $O/mat_batched.log 2>&1 || exit $?
timeout -k 10 300 python scripts/bench_materials.py --batch 1 --cpu-rows 1 > $O/mat_one.log 2>&1 || exit $?
for f in $O/bench_*.log $O/mat_*.log; do python3 -c "import json; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); r=d['roofline']; u=d.get('unbatched') or {}; print('$f', round(d['value'],1), d['ms_per_step'], r['avg_launch_ms'], r['frac'], u.get('value'), u.get('ms_per_step'))"; done
