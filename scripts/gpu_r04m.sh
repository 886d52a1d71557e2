#!/bin/bash
# r04 session M: the material kernel escape cones (parity, then A/B
# against PSRT_MAT_CONE=0).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r04m
mkdir -p $O
L=petershirleyraytracer_amd/lib
timeout -k 10 400 python -u -m pytest tests/test_gpu_materials.py -x -q --timeout 200 --timeout-method thread > $O/pytest_mat.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_mat.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for lib in libpsrt.so libpsrt_mcone0.so; do
    PSRT_LIB=$L/$lib timeout -k 10 300 python scripts/bench_materials.py --spp 10 --cpu-rows 1 > $O/mat_${lib}_$r.log 2>&1 || exit $?
    python3 -c "import json; d=json.loads([l for l in open('$O/mat_${lib}_$r.log') if l.startswith('{')][-1]); r=d['roofline']; print('mat $lib $r', round(d['value'],1), round(d['kernel_ms'],4), r['executed_box_tests_per_launch'], r.get('executed_sphere_tests_per_launch'), r.get('frac'))"
  done
done
