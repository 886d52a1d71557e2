#!/bin/bash
# r06 session ZB: what a cheaper generator would save (measurement only): the
# look-ahead trials' three PCG32 draws replaced by xorshift32 steps
# (PSRT_CHEAP_RNG_AB, different numbers, not bit-exact) against the product,
# C3 batched, three alternating rounds; kernel time per traced ray compared.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06zb
mkdir -p $O
L=petershirleyraytracer_amd/lib
for i in 1 2 3; do
  for v in base cheaprng; do
    lib=$L/libpsrt_$v.so; [ $v = base ] && lib=$L/libpsrt.so
    PSRT_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline > $O/c3_${v}_$i.log 2>&1 || exit 1
  done
done
for f in $O/c3_*.log; do python3 -c "import json; d=json.loads([l for l in open('$f') if l.startswith('{') and '\"metric\"' in l][-1]); r=d['roofline']; print('$f', d['ms_per_step'], r['avg_launch_ms'], r['rays_traced_per_launch'], round(r['avg_launch_ms']*1e6/r['rays_traced_per_launch'],4))"; done
