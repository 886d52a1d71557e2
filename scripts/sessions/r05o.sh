#!/bin/bash
# r05 session O: the launch drain walks parked rays at once (PSRT_DRAIN_WALK):
# parity tests on the variant, then C3 and the material bench, one frame per
# launch (where the drain shows) and batched, alternating with the product.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05o
mkdir -p $O
L=petershirleyraytracer_amd/lib
PSRT_LIB=$L/libpsrt_drain.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_culling.py tests/test_gpu_materials.py tests/test_gpu_sweep.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_drain.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_drain.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for v in base drain; do
    if [ $v = base ]; then E=""; else E="PSRT_LIB=$L/libpsrt_drain.so"; fi
    env $E timeout -k 10 300 python bench.py --no-cpu-baseline --batch 1 --steps 10 > $O/c3one_${v}_$i.log 2>&1 || exit $?
    env $E timeout -k 10 300 python bench.py --no-cpu-baseline > $O/c3_${v}_$i.log 2>&1 || exit $?
    env $E timeout -k 10 300 python scripts/bench_materials.py --cpu-rows 1 --batch 1 > $O/matone_${v}_$i.log 2>&1 || exit $?
    env $E timeout -k 10 300 python scripts/bench_materials.py --cpu-rows 1 > $O/mat_${v}_$i.log 2>&1 || exit $?
  done
done
for f in $O/c3*.log; do python3 -c "import json; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); print('$f', round(d['value'],1), d['ms_per_step'], d['roofline']['avg_launch_ms'])"; done
for f in $O/mat*.log; do python3 -c "import json; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); print('$f', round(d['value'],1), round(d['ms_per_step'],4), round(d['kernel_ms'],4))"; done
