#!/bin/bash
# r05 session M: the look-ahead trial queue in LDS (a two-slot ring per lane,
# PSRT_LDS_TRIALS) with 768-thread workgroups (two per CU, the scene staging
# kept), against 768-thread workgroups alone and the product; C3 bench lines
# alternating, parity through the bench's reference check and the GPU parity tests.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05m
mkdir -p $O
L=petershirleyraytracer_amd/lib
PSRT_LIB=$L/libpsrt_ldsq768.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_culling.py tests/test_gpu_sweep.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_ldsq.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_ldsq.log; [ $rc -eq 0 ] || exit $rc
PSRT_LIB=$L/libpsrt_ldsq768.so timeout -k 10 600 python bench.py > $O/bench_ldsq_ref.log 2>&1 || exit $?
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_base_$i.log 2>&1 || exit $?
  PSRT_LIB=$L/libpsrt_ldsq768.so timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_ldsq_$i.log 2>&1 || exit $?
  PSRT_LIB=$L/libpsrt_b768.so timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_b768_$i.log 2>&1 || exit $?
done
for f in $O/bench_*.log; do python3 -c "import json; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); r=d['roofline']; print('$f', round(d['value'],1), d['ms_per_step'], r['avg_launch_ms'], (d.get('parity_vs_cpu') or {}).get('fp64_bit_identical'), d['batch_check']['last_frame_equal'])"; done
