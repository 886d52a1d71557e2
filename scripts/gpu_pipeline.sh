#!/bin/bash
# Frame pipelining: C3 and a 1/8 shard at 1/2/3 frames in flight, then the
# N>1 bench loop rehearsed with 2 ranks on one GPU (gloo).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
i=0
for sh in ${SHARDS:-0/1 0/8}; do
  for d in ${DEPTHS:-1 2 3}; do
    i=$((i+1))
    E=""; [ "$sh" != "0/1" ] && E="--emulate-shard $sh"
    timeout -k 10 120 python bench.py --no-cpu-baseline --steps ${STEPS:-10} --warmup 2 --pipeline $d $E > gpurun_out/pipe_$i.log 2>&1 || exit $?
    python3 -c "import json; d=json.loads(open('gpurun_out/pipe_$i.log').read().strip().splitlines()[-1]); print('$sh depth $d', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
  done
done
PSRT_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node ${NPROC:-2} --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus ${NPROC:-2} --steps 4 --warmup 1 > gpurun_out/pipe_gloo2.log 2>&1
rc=$?; echo "gloo2 rc=$rc"; tail -1 gpurun_out/pipe_gloo2.log | cut -c1-400
exit $rc
