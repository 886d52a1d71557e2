#!/bin/bash
# r03 (session 2): GPU suite on a variant (SUITE_LIB), material kernel A/B
# (MAT_LIBS, scripts/gpu_mat_ab.sh), C3 A/B of library builds (LIBS)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r03j
O=gpurun_out/r03j
PSRT_LIB=petershirleyraytracer_amd/lib/${SUITE_LIB:-libpsrt.so} timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest ($SUITE_LIB) rc=$rc"; tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
if [ -n "$MAT_LIBS" ]; then LIBS="$MAT_LIBS" bash scripts/gpu_mat_ab.sh 2>&1 | tee $O/mat_ab.txt || exit 1; fi
ROUNDS=${ROUNDS:-3} LIBS="${LIBS:-libpsrt.so}" bash scripts/gpu_lib_ab.sh 2>&1 | tee $O/ab.txt
