#!/bin/bash
# r06 session A: the GPU suite on the round's starting tree, then the driver's
# 8-rank command rehearsed on one GPU over gloo for C3
# and C4; the JSON lines go to gpurun_out/r06_rehearsal8/.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06a
R=gpurun_out/r06_rehearsal8
mkdir -p $O $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
export PSRT_BENCH_BACKEND=gloo MASTER_ADDR=127.0.0.1 OMP_NUM_THREADS=2
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 8 --config c3 > $R/c3_n8.log 2>&1 || { tail -30 $R/c3_n8.log; exit 1; }
grep '^{' $R/c3_n8.log | tail -1 > $R/c3_n8.json
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29532 bench.py --gpus 8 --config c4 --steps 1 --warmup 0 > $R/c4_n8.log 2>&1 || { tail -30 $R/c4_n8.log; exit 1; }
grep '^{' $R/c4_n8.log | tail -1 > $R/c4_n8.json
python3 - <<'PY'
import json
for c in ("c3", "c4"):
    d = json.load(open(f"gpurun_out/r06_rehearsal8/{c}_n8.json"))
    print(c, d["value"], d["ms_per_step"], len(d["per_rank"]), d["parity_vs_cpu"].get("checked"), d["parity_vs_cpu"].get("ranks_covered"), d["batch_check"].get("all_ranks_equal"))
PY
