#!/bin/bash
# r06 session ZI: with frames in flight, does the launch tail's raised issue
# priority still pay? C3 one frame per launch, two in flight, with and without
# it (RT_FLAG_NO_TAIL_PRIORITY), three alternating rounds.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06zi
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --batch 1 --pipeline 2 > $O/c3p2_tail_$i.log 2>&1 || exit 1
  timeout -k 10 200 python bench.py --no-cpu-baseline --batch 1 --pipeline 2 --no-tail-priority > $O/c3p2_notail_$i.log 2>&1 || exit 1
done
for f in $O/c3*.log; do python3 -c "import json; d=json.loads([l for l in open('$f') if l.startswith('{') and '\"metric\"' in l][-1]); print('$f', d['value'], d['ms_per_step'], d['tail_priority'])"; done
