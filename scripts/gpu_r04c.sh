#!/bin/bash
# r04 session C: the GPU suite on the FP32 pre-reject build (both kernels),
# the material kernel's pre-reject A/B, the C3 section census (diagnostic
# stamps build) and a re-sweep of the refill / walk-batch knobs.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r04c
mkdir -p $O
L=petershirleyraytracer_amd/lib
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for lib in libpsrt.so libpsrt_matnopre.so; do
    PSRT_LIB=$L/$lib timeout -k 10 300 python scripts/bench_materials.py --spp 10 --cpu-rows 1 > $O/mat_${lib}_$r.log 2>&1 || exit $?
    python3 -c "import json; d=json.loads([l for l in open('$O/mat_${lib}_$r.log') if l.startswith('{')][-1]); print('mat $lib $r', round(d['value'],1), round(d['kernel_ms'],4), d['roofline']['executed_sphere_tests_per_launch'], d['roofline']['frac'])"
  done
done
timeout -k 10 300 python scripts/stamps_c3.py > $O/stamps_c3.log 2>&1 || exit $?
tail -4 $O/stamps_c3.log
for r in 1 2; do
  for lib in libpsrt.so libpsrt_r12.so libpsrt_r20.so libpsrt_b20.so libpsrt_b28.so; do
    PSRT_LIB=$L/$lib timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/c3_${lib}_$r.log 2>&1 || exit $?
    python3 -c "import json; d=json.loads([l for l in open('$O/c3_${lib}_$r.log') if l.startswith('{')][-1]); print('c3 $lib $r', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
  done
done
