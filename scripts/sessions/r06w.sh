#!/bin/bash
# r06 session W: the 8-rank C3 rehearsal again with one context per rank
# (session V: 7250-7470 Msamples/s with two, against 8146 before frames in
# flight), twice, and C4 once.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06w
mkdir -p $O
export PSRT_BENCH_BACKEND=gloo MASTER_ADDR=127.0.0.1 OMP_NUM_THREADS=2
for i in 1 2; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 2956$i bench.py --gpus 8 --config c3 > $O/c3_n8_$i.log 2>&1 || { tail -30 $O/c3_n8_$i.log; exit 1; }
  grep '^{' $O/c3_n8_$i.log | tail -1 > $O/c3_n8_$i.json
  python3 -c "import json; d=json.load(open('$O/c3_n8_$i.json')); print('c3 n8', d['value'], d['ms_per_step'], [round(r['kernel_ms'],2) for r in d['per_rank']], d['parity_vs_cpu'].get('ranks_covered'), d['batch_check'].get('all_ranks_equal'), d.get('host_frame_check'))"
done
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29569 bench.py --gpus 8 --config c4 --steps 1 --warmup 0 > $O/c4_n8.log 2>&1 || { tail -30 $O/c4_n8.log; exit 1; }
grep '^{' $O/c4_n8.log | tail -1 > $O/c4_n8.json
python3 -c "import json; d=json.load(open('$O/c4_n8.json')); print('c4 n8', d['value'], d['ms_per_step'], d['parity_vs_cpu'].get('ranks_covered'), d['batch_check'].get('all_ranks_equal'), d.get('host_frame_check'))"
