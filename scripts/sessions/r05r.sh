#!/bin/bash
# r05 session R: the material walk batch (tuning knob mat_batch) re-swept on
# the r05 kernel, 10 frames per launch, two rounds.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05r
mkdir -p $O
for i in 1 2; do
  for b in 16 32 48 64 96; do
    timeout -k 10 300 python scripts/bench_materials.py --cpu-rows 1 --tune mat_batch=$b > $O/mat_b${b}_$i.log 2>&1 || exit $?
  done
done
for f in $O/mat*.log; do python3 -c "import json; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); print('$f', round(d['value'],1), round(d['kernel_ms'],4), d['unbatched']['kernel_ms'])"; done
