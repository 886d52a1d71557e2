#!/bin/bash
# r03 (session 2): GPU suite on the inline list records, then a C3 A/B of
# library builds (scripts/gpu_lib_ab.sh)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r03h
O=gpurun_out/r03h
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
ROUNDS=${ROUNDS:-3} LIBS="${LIBS:-libpsrt_old.so libpsrt.so}" bash scripts/gpu_lib_ab.sh 2>&1 | tee $O/ab.txt
