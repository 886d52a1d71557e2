#!/bin/bash
# r04 session H: one psrt_reduce launch per multi-frame batch: parity subset,
# C3 and the 1/8 shard A/B against the per-frame reduce launches (prevred).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r04h
mkdir -p $O
L=petershirleyraytracer_amd/lib
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_context.py tests/test_gpu_bench.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for lib in libpsrt.so libpsrt_prevred.so; do
    PSRT_LIB=$L/$lib timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/c3_${lib}_$r.log 2>&1 || exit $?
    PSRT_LIB=$L/$lib timeout -k 10 300 python bench.py --emulate-shard 0/8 --steps 20 --warmup 5 > $O/s8_${lib}_$r.log 2>&1 || exit $?
    python3 -c "
import json
for f in ['$O/c3_${lib}_$r.log','$O/s8_${lib}_$r.log']:
    d=json.loads([l for l in open(f) if l.startswith('{')][-1]); print(f.split('/')[-1], d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
  done
done
