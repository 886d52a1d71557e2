#!/bin/bash
# material tests, then the material bench over settings "VAR=value ..." (SETTINGS)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_materials.py > gpurun_out/mat.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 gpurun_out/mat.log; [ $rc -eq 0 ] || exit $rc
i=0
for kv in $SETTINGS; do
  i=$((i+1))
  env $kv timeout -k 10 300 python -u scripts/bench_materials.py --cpu-rows 1 > gpurun_out/bme_$i.log 2>&1 || exit $?
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/bme_$i.log') if l.startswith('{')][-1]); r=d['roofline']; print('$kv', round(d['value'],1), round(d['kernel_ms'],4), r['frac'], r['executed_box_tests_per_launch'])"
done
