#!/bin/bash
# sharded queue heads: GPU suite, then A/B (cur vs q1) on C1, C2, C3 and a 1/64 shard
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for c in ${CFGS:-c1 c2 c3}; do
  echo "== $c"; CONFIG=$c LIBS="cur q1" ROUNDS=2 STEPS=20 bash scripts/gpu_variants.sh || exit $?
done
echo "== c3 1/64 shard"; CONFIG=c3 LIBS="cur q1" ROUNDS=2 STEPS=20 BENCH_ARGS="--emulate-shard 0/64 --scaling strong" bash scripts/gpu_variants.sh || exit $?
