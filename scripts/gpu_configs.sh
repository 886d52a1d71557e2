#!/bin/bash
# all bench configurations at 1 GPU + the torchrun (RCCL, world 1) path + profiles
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for c in c1 c2 c4; do
  timeout -k 10 600 python bench.py --config $c --steps 2 --warmup 1 > gpurun_out/bench_$c.log 2>&1
  rc=$?; echo "bench $c rc=$rc"; tail -1 gpurun_out/bench_$c.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 600 python bench.py --config c5 --steps 1 --warmup 0 --cpu-seconds 8 > gpurun_out/bench_c5.log 2>&1
rc=$?; echo "bench c5 rc=$rc"; tail -1 gpurun_out/bench_c5.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 1 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_torchrun1.log 2>&1
rc=$?; echo "torchrun rc=$rc"; tail -1 gpurun_out/bench_torchrun1.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
CONFIG=c3 STEPS=2 bash scripts/gpu_profile.sh
