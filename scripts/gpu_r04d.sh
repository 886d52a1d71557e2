#!/bin/bash
# r04 session D: parity subset on the default build (FP32 far-origin test),
# then C3 A/B: FP32 far test on / off, a depth-3 trial queue (2 + 1 or 2 + 0
# rounds); the material kernel with priorities and no pre-reject.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r04d
mkdir -p $O
L=petershirleyraytracer_amd/lib
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_culling.py tests/test_gpu_culling_kat.py tests/test_gpu_materials.py -x -q --timeout 300 --timeout-method thread > $O/pytest_subset.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_subset.log; [ $rc -eq 0 ] || exit $rc
for lib in libpsrt_q3.so libpsrt_q3e0.so; do
  PSRT_LIB=$L/$lib timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -k "full_frames or fixtures or trace" --timeout 300 --timeout-method thread > $O/pytest_$lib.log 2>&1
  rc=$?; echo "pytest $lib rc=$rc"; tail -1 $O/pytest_$lib.log; [ $rc -eq 0 ] || exit $rc
done
for r in 1 2; do
  for lib in libpsrt.so libpsrt_nofar.so libpsrt_q3.so libpsrt_q3e0.so; do
    PSRT_LIB=$L/$lib timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/c3_${lib}_$r.log 2>&1 || exit $?
    python3 -c "import json; d=json.loads([l for l in open('$O/c3_${lib}_$r.log') if l.startswith('{')][-1]); print('c3 $lib $r', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['batch_check']['last_frame_equal'])"
  done
done
for r in 1 2; do
  timeout -k 10 300 python scripts/bench_materials.py --spp 10 --cpu-rows 1 > $O/mat_$r.log 2>&1 || exit $?
  python3 -c "import json; d=json.loads([l for l in open('$O/mat_$r.log') if l.startswith('{')][-1]); print('mat $r', round(d['value'],1), round(d['kernel_ms'],4), d['roofline']['frac'])"
done
