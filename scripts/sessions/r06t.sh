#!/bin/bash
# r06 session T: batched frames as a chain of smaller launches, two in flight
# (bench candidates b/2, b/4 against one launch of b): the default C3 line,
# the 7/8 shard, C2 and C1, each against --no-chain, alternating.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06t
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench.py tests/test_gpu_inflight.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --no-cpu-baseline > $O/c3_chain_$i.log 2>&1 || exit 1
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-chain > $O/c3_one_$i.log 2>&1 || exit 1
  timeout -k 10 200 python bench.py --no-cpu-baseline --emulate-shard 7/8 > $O/s78_chain_$i.log 2>&1 || exit 1
  timeout -k 10 200 python bench.py --no-cpu-baseline --emulate-shard 7/8 --no-chain > $O/s78_one_$i.log 2>&1 || exit 1
done
for c in c2 c1; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --config $c > $O/${c}_chain.log 2>&1 || exit 1
  timeout -k 10 200 python bench.py --no-cpu-baseline --config $c --no-chain > $O/${c}_one.log 2>&1 || exit 1
done
for f in $O/c*.log $O/s78*.log; do python3 -c "import json; d=json.loads([l for l in open('$f') if l.startswith('{') and '\"metric\"' in l][-1]); print('$f', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['frames_per_launch'], d['frames_in_flight'], d.get('depth_tuning_ms'), d['batch_check']['last_frame_equal'])"; done
