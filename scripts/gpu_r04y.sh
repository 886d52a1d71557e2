#!/bin/bash
# r04 session Y: the trace loop's thresholds re-swept on the final kernel:
# walk tail (PSRT_WALK_TAIL 2 / 6, default 4), walk batch (20 / 28, default
# 24), refill (14 / 18, default 16). C3, 20 steps, psrt_trace ms per frame.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r04y
mkdir -p $O
L=petershirleyraytracer_amd/lib
for r in 1 2; do
  for lib in libpsrt.so libpsrt_t2.so libpsrt_t6.so libpsrt_wb20.so libpsrt_wb28.so libpsrt_rf14.so libpsrt_rf18.so; do
    PSRT_LIB=$L/$lib timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/c3_${lib}_$r.log 2>&1 || exit $?
    python3 -c "import json; d=json.loads([l for l in open('$O/c3_${lib}_$r.log') if l.startswith('{')][-1]); print('c3 $lib $r', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['batch_check']['last_frame_equal'])"
  done
done
