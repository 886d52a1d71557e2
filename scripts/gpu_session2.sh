#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
bash scripts/gpu_check.sh || exit $?
for c in c1 c2; do
  timeout -k 10 600 python bench.py --config $c --steps 3 --no-cpu-baseline > gpurun_out/bench_$c.log 2>&1
  rc=$?; echo "bench $c rc=$rc"; tail -1 gpurun_out/bench_$c.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
done
CONFIG=c3 bash scripts/gpu_profile.sh
