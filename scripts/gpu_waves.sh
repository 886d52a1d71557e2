#!/bin/bash
# default knobs at G=1/8/64, then the diagnostic wave timeline (PSRT_STAMPS)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
SHARDS="${SHARDS:-0/1 0/8 0/64}" bash scripts/gpu_knobs.sh || exit $?
for sh in ${SHARDS:-0/1 0/8 0/64}; do
  E=""; [ "$sh" != "0/1" ] && E="--emulate-shard $sh"
  PSRT_STAMPS=1 timeout -k 10 120 python bench.py --no-cpu-baseline --steps 1 --warmup 1 $E > gpurun_out/waves.log 2>&1 || exit $?
  echo "$sh"; grep psrt_waves gpurun_out/waves.log | tail -1
done
