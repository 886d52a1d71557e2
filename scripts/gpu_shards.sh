#!/bin/bash
# Per-rank step time of the multi-GPU bench, emulated on one GPU: rank R of G
# renders only its interleaved rows (bench.py --emulate-shard R/G). The
# slowest rank bounds the N-GPU step (plus the uint8 gather).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
CONFIG=${CONFIG:-c3}
STEPS=${STEPS:-10}
timeout -k 10 300 python bench.py --config $CONFIG --steps $STEPS --warmup 2 --no-cpu-baseline > gpurun_out/shard_1.log 2>&1 || exit $?
python3 -c "import json; d=json.loads(open('gpurun_out/shard_1.log').read().strip().splitlines()[-1]); print('G=1', d['ms_per_step'], d['roofline']['avg_launch_ms'])"
for G in ${GS:-2 4 8}; do
  for R in $(seq 0 $((G-1))); do
    timeout -k 10 300 python bench.py --config $CONFIG --steps $STEPS --warmup 2 --emulate-shard $R/$G > gpurun_out/shard_${R}_$G.log 2>&1 || exit $?
    python3 -c "import json; d=json.loads(open('gpurun_out/shard_${R}_$G.log').read().strip().splitlines()[-1]); print('G=$G R=$R', d['ms_per_step'], d['roofline']['avg_launch_ms'])"
  done
done
