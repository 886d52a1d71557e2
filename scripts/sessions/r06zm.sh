#!/bin/bash
# r06 session ZM: the per-sample seeding with 32-bit operations (lowbias32 per
# word, full avalanche; measurement build PSRT_SEED32_AB, not the contract)
# against splitmix64, C3 batched, three alternating rounds.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06zm
mkdir -p $O
L=petershirleyraytracer_amd/lib
for i in 1 2 3; do
  for v in base seed32; do
    lib=$L/libpsrt_$v.so; [ $v = base ] && lib=$L/libpsrt.so
    PSRT_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline > $O/c3_${v}_$i.log 2>&1 || exit 1
  done
done
for f in $O/c3_*.log; do python3 -c "import json; d=json.loads([l for l in open('$f') if l.startswith('{') and '\"metric\"' in l][-1]); r=d['roofline']; print('$f', d['ms_per_step'], r['avg_launch_ms'], r['rays_traced_per_launch'])"; done
