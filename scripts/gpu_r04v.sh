#!/bin/bash
# r04 session V: work-queue shape for short launches (the strong 1/8 shard,
# 20 frames per launch = 24 M units): PSRT_QUEUE_K (tickets per wave per
# phase) and PSRT_QUEUE_D (first ticket <= units / (D x waves)).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r04v
mkdir -p $O
for r in ${ROUNDS:-1 2}; do
  for kd in ${KDS:-"1 4" "2 4" "1 2" "2 2" "1 8" "0.5 4"}; do
    set -- $kd
    tag="k$1_d$2"
    PSRT_QUEUE_K=$1 PSRT_QUEUE_D=$2 timeout -k 10 300 python bench.py --emulate-shard 7/8 --steps 20 --warmup 5 --no-cpu-baseline > $O/s8_${tag}_$r.log 2>&1 || exit $?
    python3 -c "import json; d=json.loads([l for l in open('$O/s8_${tag}_$r.log') if l.startswith('{')][-1]); print('s8 7/8 $tag $r', d['ms_per_step'], d['roofline']['avg_launch_ms'])"
  done
done
