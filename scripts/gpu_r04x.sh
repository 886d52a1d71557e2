#!/bin/bash
# r04 session X: psrt_reduce forms a sample's colour without branches when
# every k < 1000 (ReduceArgs::fast_k): parity subset, then C3 and the 7/8
# shard A/B against the previous build (libpsrt_head.so).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r04x
mkdir -p $O
L=petershirleyraytracer_amd/lib
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_context.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for lib in libpsrt.so libpsrt_head.so; do
    PSRT_LIB=$L/$lib timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/c3_${lib}_$r.log 2>&1 || exit $?
    PSRT_LIB=$L/$lib timeout -k 10 300 python bench.py --emulate-shard 7/8 --steps 20 --warmup 5 --no-cpu-baseline > $O/s8_${lib}_$r.log 2>&1 || exit $?
    python3 -c "
import json
for f in ['$O/c3_${lib}_$r.log','$O/s8_${lib}_$r.log']:
    d=json.loads([l for l in open(f) if l.startswith('{')][-1]); print(f.split('/')[-1], d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['batch_check']['last_frame_equal'] if 'batch_check' in d else '')"
  done
done
