#!/bin/bash
# material tests + material bench (BVH in LDS or not) + C3 knob sweep
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_materials.py > gpurun_out/mat.log 2>&1 || { tail -20 gpurun_out/mat.log; exit 1; }
tail -1 gpurun_out/mat.log
for l in 0 1; do
  PSRT_MAT_LDS=$l timeout -k 10 200 python -u scripts/bench_materials.py --spp 10 --cpu-rows 1 > gpurun_out/bm_lds$l.log 2>&1 || exit $?
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/bm_lds$l.log') if l.startswith('{')][-1]); print('mat lds $l', round(d['value'],1), d['kernel_ms'])"
done
KNOBS="${KNOBS:-PSRT_REFILL_MIN=8 PSRT_REFILL_MIN=10 PSRT_REFILL_MIN=12 PSRT_BATCH=16 PSRT_BATCH=18 PSRT_BATCH=20}" bash scripts/gpu_knobs_r03.sh
