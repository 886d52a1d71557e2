#!/bin/bash
# r04 session U: one 64-B LDS record per sphere (sphere, FP32 pre-reject sphere,
# neighbour record, 1/r: one base register, one index computation)
# instead of four arrays: parity subset, then C3 A/B against
# the previous build (libpsrt_head.so).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r04u
mkdir -p $O
L=petershirleyraytracer_amd/lib
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_culling.py tests/test_gpu_culling_kat.py tests/test_gpu_context.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for lib in libpsrt.so libpsrt_head.so; do
    PSRT_LIB=$L/$lib timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/c3_${lib}_$r.log 2>&1 || exit $?
    python3 -c "import json; d=json.loads([l for l in open('$O/c3_${lib}_$r.log') if l.startswith('{')][-1]); print('c3 $lib $r', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['batch_check']['last_frame_equal'])"
  done
done
