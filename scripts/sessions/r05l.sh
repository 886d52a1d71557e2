#!/bin/bash
# r05 session L: the final tree: GPU suite, smoke, the default bench line
# three times, one frame per launch, the material bench (batched and one
# frame per launch).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${SESSION_OUT:-r05l}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > $O/bench_default.log 2>&1 || exit $?
for i in 2 3; do timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_c3_$i.log 2>&1 || exit $?; done
timeout -k 10 300 python bench.py --no-cpu-baseline --batch 1 > $O/bench_c3_batch1.log 2>&1 || exit $?
timeout -k 10 300 python scripts/bench_materials.py > $O/mat_batched.log 2>&1 || exit $?
timeout -k 10 300 python scripts/bench_materials.py --batch 1 --cpu-rows 1 > $O/mat_one.log 2>&1 || exit $?
for f in $O/bench_*.log $O/mat_*.log; do python3 -c "import json; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); r=d['roofline']; print('$f', round(d['value'],1), d['ms_per_step'], r['avg_launch_ms'], r['frac'], (r.get('valu_issue') or {}).get('lane_utilisation'))"; done
