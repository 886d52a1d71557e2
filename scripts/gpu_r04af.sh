#!/bin/bash
# r04 session AF: tickets hand out the launch's units from the last one
# (PSRT_UNIT_REVERSE=1: each frame's top rows, the sky, go last) against the
# forward order; parity of the reversed build, then C3 and the 7/8 and 0/8
# shards, two rounds.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r04af
mkdir -p $O
L=petershirleyraytracer_amd/lib
PSRT_LIB=$L/libpsrt_rev.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/parity_rev.log 2>&1 || { tail -20 $O/parity_rev.log; exit 1; }
tail -2 $O/parity_rev.log
for r in 1 2; do
  for lib in libpsrt.so libpsrt_rev.so; do
    for sh in "" "--emulate-shard 7/8" "--emulate-shard 0/8"; do
      n=$(echo "c3$sh" | tr -d ' -/')
      PSRT_LIB=$L/$lib timeout -k 10 300 python bench.py $sh --steps 20 --warmup 5 --no-cpu-baseline > $O/${n}_${lib}_$r.log 2>&1 || exit $?
      python3 -c "
import json
d=json.loads([l for l in open('$O/${n}_${lib}_$r.log') if l.startswith('{')][-1]); print('${n} $lib $r', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['unbatched']['kernel_ms'], d['batch_check']['last_frame_equal'], d['batch_check']['first_frame_equal_counting_kernel'])"
    done
  done
done
