#!/bin/bash
# r06 session I: frames assembled in shared page-locked host memory (bench
# --assemble host, rt_context_set_row_pitch, rt_host_register): their GPU
# tests, then the driver's 8-rank command rehearsed again on one GPU for C3
# and C4 with --assemble host (the default on one node) and gather.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06i
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_host.py tests/test_gpu_bench.py tests/test_gpu_group.py tests/test_host_api.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
export PSRT_BENCH_BACKEND=gloo MASTER_ADDR=127.0.0.1 OMP_NUM_THREADS=2
for a in host gather; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 2954${#a} bench.py --gpus 8 --config c3 --assemble $a > $O/c3_n8_$a.log 2>&1 || { tail -30 $O/c3_n8_$a.log; exit 1; }
done
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 8 --config c4 --steps 1 --warmup 0 > $O/c4_n8_host.log 2>&1 || { tail -30 $O/c4_n8_host.log; exit 1; }
ls /dev/shm | grep psrt_ || echo "no psrt segments left in /dev/shm"
for f in $O/c*_n8_*.log; do python3 -c "
import json; d=json.loads([l for l in open('$f') if l.startswith('{') and '\"metric\"' in l][-1])
print('$f', d['value'], d['ms_per_step'], d['frame_to_host'], len(d['per_rank']), d['parity_vs_cpu'].get('fp64_bit_identical'), d['parity_vs_cpu'].get('ranks_covered'), d['batch_check'].get('all_ranks_equal'), d.get('host_frame_check'))"; done
