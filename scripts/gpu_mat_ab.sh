#!/bin/bash
# material tests, then the material bench for the default lib and A/B libs
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_materials.py > gpurun_out/mat.log 2>&1 || { tail -30 gpurun_out/mat.log; exit 1; }
tail -1 gpurun_out/mat.log
for lib in ${LIBS:-libpsrt.so}; do for l in ${LDS:-1}; do
  PSRT_LIB=petershirleyraytracer_amd/lib/$lib PSRT_MAT_LDS=$l timeout -k 10 200 python -u scripts/bench_materials.py --spp 10 --cpu-rows 1 > gpurun_out/bm_$lib.$l.log 2>&1 || exit $?
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/bm_$lib.$l.log') if l.startswith('{')][-1]); print('mat $lib lds $l', round(d['value'],1), d['kernel_ms'])"
done; done
