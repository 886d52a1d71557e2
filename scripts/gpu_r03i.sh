#!/bin/bash
# r03 (session 2): GPU suite on a variant build (PSRT_LIB), then a C3 A/B of
# library builds (scripts/gpu_lib_ab.sh)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r03i
O=gpurun_out/r03i
PSRT_LIB=petershirleyraytracer_amd/lib/${SUITE_LIB:-libpsrt.so} timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest ($SUITE_LIB) rc=$rc"; tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
ROUNDS=${ROUNDS:-3} LIBS="${LIBS:-libpsrt.so}" bash scripts/gpu_lib_ab.sh 2>&1 | tee $O/ab.txt
