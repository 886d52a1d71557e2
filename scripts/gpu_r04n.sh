#!/bin/bash
# r04 session N: camera-ray lists through the lens in the material kernel,
# again, now beside the batched walk (parity, then A/B against
# PSRT_NO_CAMLIST=1), and 4 waves per SIMD asked of the register allocator
# (PSRT_MAT_WAVES=4: up to 128 VGPRs; LDS already limits the kernel to 4).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r04n
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_materials.py -x -q --timeout 200 --timeout-method thread > $O/pytest_mat.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_mat.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for v in list nolist mw4; do
    if [ $v = nolist ]; then export PSRT_NO_CAMLIST=1; else unset PSRT_NO_CAMLIST; fi
    if [ $v = mw4 ]; then export PSRT_LIB=petershirleyraytracer_amd/lib/libpsrt_mw4.so; else unset PSRT_LIB; fi
    timeout -k 10 300 python scripts/bench_materials.py --spp 10 --cpu-rows 1 > $O/mat_${v}_$r.log 2>&1 || exit $?
    python3 -c "import json; d=json.loads([l for l in open('$O/mat_${v}_$r.log') if l.startswith('{')][-1]); r=d['roofline']; print('mat $v $r', round(d['value'],1), round(d['kernel_ms'],4), r['executed_box_tests_per_launch'], r.get('executed_sphere_tests_per_launch'), r.get('frac'))"
  done
done
