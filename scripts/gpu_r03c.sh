#!/bin/bash
# r03: rocprofv3 trace + PMC passes of C3 (summary filtered to the timed kernel),
# then emulated per-rank shards: C4 strong 1/8 (ranks 0 and 7), C3 strong 1/2, 1/4, 1/8.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
CONFIG=c3 STEPS=3 bash scripts/gpu_profile.sh || exit $?
for s in "c4 0/8" "c4 7/8" "c3 0/2" "c3 1/2" "c3 0/4" "c3 3/4" "c3 0/8" "c3 7/8"; do
  set -- $s
  timeout -k 10 300 python bench.py --config $1 --emulate-shard $2 --steps 10 --warmup 2 > gpurun_out/shard_${1}_${2/\//of}.log 2>&1
  rc=$?; echo "shard $1 $2 rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c4.log 2>&1
echo "c4 rc=$?"
