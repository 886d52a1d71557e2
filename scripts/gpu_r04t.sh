#!/bin/bash
# r04 session T: compiler scheduling variants of the same source
# (PSRT_HIPCC_FLAGS): AMDGPU register-pressure trackers, max-ilp strategy
# (gcn-iterative-ilp crashes the device compiler); parity subset on the first,
# then C3 A/B.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r04t
mkdir -p $O
L=petershirleyraytracer_amd/lib
PSRT_LIB=$L/libpsrt_ftrk.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_culling_kat.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for lib in libpsrt.so libpsrt_ftrk.so libpsrt_filp.so; do
    PSRT_LIB=$L/$lib timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/c3_${lib}_$r.log 2>&1 || exit $?
    python3 -c "import json; d=json.loads([l for l in open('$O/c3_${lib}_$r.log') if l.startswith('{')][-1]); print('c3 $lib $r', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['batch_check']['last_frame_equal'])"
  done
done
