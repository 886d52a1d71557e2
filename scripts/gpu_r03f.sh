#!/bin/bash
# materials: lens camera lists + counting variant + CLI book scene (GPU tests),
# then the materials bench with and without the lists, and its PMC passes.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_materials.py > gpurun_out/mat.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/mat.log; [ $rc -eq 0 ] || exit $rc
for cl in 0 1; do
  if [ $cl -eq 1 ]; then export PSRT_NO_CAMLIST=1; fi
  timeout -k 10 300 python -u scripts/bench_materials.py --cpu-rows 1 > gpurun_out/bm_cl$cl.log 2>&1 || exit $?
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/bm_cl$cl.log') if l.startswith('{')][-1]); print('no_camlist=$cl', round(d['value'],1), d['kernel_ms'], d['roofline']['frac'])"
done
unset PSRT_NO_CAMLIST
bash scripts/gpu_mat_pmc.sh
