#!/bin/bash
# r05 session Q: the material walk reads both successors of a node before its
# slab test (PSRT_MAT_PREFETCH): material parity tests on the variant, then
# the material bench alternating with the product.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05q
mkdir -p $O
L=petershirleyraytracer_amd/lib
PSRT_LIB=$L/libpsrt_mpf.so timeout -k 10 600 python -u -m pytest tests/test_gpu_materials.py tests/test_gpu_sweep.py tests/test_gpu_knobs.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_mpf.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_mpf.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  timeout -k 10 300 python scripts/bench_materials.py --cpu-rows 1 > $O/mat_base_$i.log 2>&1 || exit $?
  PSRT_LIB=$L/libpsrt_mpf.so timeout -k 10 300 python scripts/bench_materials.py --cpu-rows 1 > $O/mat_mpf_$i.log 2>&1 || exit $?
done
for f in $O/mat*.log; do python3 -c "import json; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); print('$f', round(d['value'],1), round(d['ms_per_step'],4), round(d['kernel_ms'],4), d['unbatched']['kernel_ms'])"; done
