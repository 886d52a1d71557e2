#!/bin/bash
# r05 session F: the material kernel's direction lists (MatArgs::dl). The
# material GPU tests (parity with and without the lists), the new culling /
# RCCL tests, then the material bench A/B (lists on / off, batched and one
# frame per launch).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05f
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_culling.py -k sky -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python scripts/bench_materials.py --cpu-rows 1 > $O/mat_dl_$i.log 2>&1 || exit $?
  timeout -k 10 300 python scripts/bench_materials.py --cpu-rows 1 --tune no_dirlist=1 > $O/mat_nodl_$i.log 2>&1 || exit $?
done
timeout -k 10 300 python scripts/bench_materials.py --cpu-rows 1 --batch 1 > $O/mat_dl_one.log 2>&1 || exit $?
timeout -k 10 300 python scripts/bench_materials.py --cpu-rows 1 --batch 1 --tune no_dirlist=1 > $O/mat_nodl_one.log 2>&1 || exit $?
for f in $O/mat_*.log; do python3 -c "import json; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); r=d['roofline']; print('$f', round(d['value'],1), round(d['kernel_ms'],4), r['frac'], r['box_tests_evaluated_per_launch'], r['full_sphere_tests_per_launch'], d.get('unbatched'))"; done
