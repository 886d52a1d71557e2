#!/bin/bash
# r05 session K: emulated strong-scaling shards of C3 (every rank of G = 2, 4,
# 8) and C4 (ranks 0 and 7 of 8) on one GPU, and the C3 line again.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05k
mkdir -p $O
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_c3.log 2>&1 || exit $?
for G in 2 4 8; do
  for ((R=0; R<G; R++)); do
    timeout -k 10 300 python bench.py --no-cpu-baseline --emulate-shard $R/$G > $O/shard_c3_${R}_of_${G}.log 2>&1 || exit $?
  done
  echo "G=$G done"
done
for R in 0 7; do
  timeout -k 10 600 python bench.py --no-cpu-baseline --config c4 --emulate-shard $R/8 > $O/shard_c4_${R}_of_8.log 2>&1 || exit $?
done
timeout -k 10 600 python bench.py --no-cpu-baseline --config c4 > $O/bench_c4.log 2>&1 || exit $?
for f in $O/*.log; do python3 -c "import json; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); print('$f', round(d['value'],1), d['ms_per_step'], d['roofline']['avg_launch_ms'])"; done
