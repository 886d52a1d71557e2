#!/bin/bash
# materials: GPU tests, the bench line, then its PMC passes
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_materials.py > gpurun_out/mat.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/mat.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_mat_pmc.sh || exit $?
python3 scripts/summarize_mat_pmc.py gpurun_out/prof_mat_pmc > gpurun_out/pmc_mat_summary.txt 2>&1
timeout -k 10 300 python -u scripts/bench_materials.py > gpurun_out/bm_final.log 2>&1 || exit $?
python3 -c "import json; d=json.loads([l for l in open('gpurun_out/bm_final.log') if l.startswith('{')][-1]); print(round(d['value'],1), d['kernel_ms'], d['roofline'])"
