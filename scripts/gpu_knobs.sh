#!/bin/bash
# bench sweep over env knobs x emulated shards (kernel time only)
# KNOBS="PSRT_TAIL_WINDOWS=0 PSRT_TAIL_WINDOWS=2,PSRT_BATCH=24" SHARDS="0/1 0/8"
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
i=0
for sh in ${SHARDS:-0/1}; do
  for kv in ${KNOBS:-DEFAULT=1}; do
    i=$((i+1))
    E=""; [ "$sh" != "0/1" ] && E="--emulate-shard $sh"
    env ${kv//,/ } timeout -k 10 120 python bench.py --no-cpu-baseline --steps ${STEPS:-10} --warmup 2 $E ${BENCH_ARGS} > gpurun_out/knob_$i.log 2>&1 || exit $?
    python3 -c "import json; d=json.loads(open('gpurun_out/knob_$i.log').read().strip().splitlines()[-1]); print('$sh $kv', d['ms_per_step'], d['roofline']['avg_launch_ms'])"
  done
done
