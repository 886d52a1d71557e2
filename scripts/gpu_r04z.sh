#!/bin/bash
# r04 session Z: walk tail 4 (default) / 6 / 8, three rounds, C3 and the 7/8
# shard.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r04z
mkdir -p $O
L=petershirleyraytracer_amd/lib
for r in 1 2 3; do
  for lib in libpsrt.so libpsrt_t6.so libpsrt_t8.so; do
    PSRT_LIB=$L/$lib timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/c3_${lib}_$r.log 2>&1 || exit $?
    PSRT_LIB=$L/$lib timeout -k 10 300 python bench.py --emulate-shard 7/8 --steps 20 --warmup 5 --no-cpu-baseline > $O/s8_${lib}_$r.log 2>&1 || exit $?
    python3 -c "
import json
for f in ['$O/c3_${lib}_$r.log','$O/s8_${lib}_$r.log']:
    d=json.loads([l for l in open(f) if l.startswith('{')][-1]); print(f.split('/')[-1], d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
  done
done
