#!/bin/bash
# r06 session ZN: the guided queue's shape (runtime knobs queue_k, queue_d)
# re-swept on the final kernel, C3 batched and one frame per launch (two in
# flight), two alternating rounds.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06zn
mkdir -p $O
for i in 1 2; do
  for t in "" "queue_k=1" "queue_k=3" "queue_d=1" "queue_d=4"; do
    n=${t:-default}; n=${n/=/}
    timeout -k 10 200 python bench.py --no-cpu-baseline ${t:+--tune $t} > $O/c3_${n}_$i.log 2>&1 || exit 1
    timeout -k 10 200 python bench.py --no-cpu-baseline --batch 1 --pipeline 2 ${t:+--tune $t} > $O/c3one_${n}_$i.log 2>&1 || exit 1
  done
done
for f in $O/c3*.log; do python3 -c "import json; d=json.loads([l for l in open('$f') if l.startswith('{') and '\"metric\"' in l][-1]); print('$f', d['ms_per_step'], d['roofline']['avg_launch_ms'])"; done
