#!/bin/bash
# r06 session P: session O again with psrt_reduce_lean at issue priority 3
# (beside the trace, whose waves run at 1-3, a priority-0 reduce took the
# whole next trace launch: 12 ms).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06p
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_inflight.py tests/test_gpu_knobs.py -x -v --timeout 200 --timeout-method thread > $O/pytest_inflight.log 2>&1 || { tail -40 $O/pytest_inflight.log; exit 1; }
tail -1 $O/pytest_inflight.log
for d in 2 3; do
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/p${d}l -o run -- python3 bench.py --batch 1 --pipeline $d --steps 10 --warmup 2 --no-cpu-baseline > $O/trace_p${d}l.log 2>&1 || { tail -20 $O/trace_p${d}l.log; exit 1; }
done
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --batch 1 --pipeline 1 > $O/c3p1_$i.log 2>&1 || exit 1
  for d in 2 3; do
    timeout -k 10 200 python bench.py --no-cpu-baseline --batch 1 --pipeline $d > $O/c3p${d}l_$i.log 2>&1 || exit 1
    timeout -k 10 200 python bench.py --no-cpu-baseline --batch 1 --pipeline $d --no-lean-reduce > $O/c3p${d}n_$i.log 2>&1 || exit 1
  done
done
timeout -k 10 200 python bench.py --no-cpu-baseline --batch 1 > $O/c3auto.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline > $O/c3default.log 2>&1 || exit 1
for f in $O/c3*.log $O/trace_*.log; do python3 -c "import json; d=json.loads([l for l in open('$f') if l.startswith('{') and '\"metric\"' in l][-1]); u=d.get('unbatched') or {}; print('$f', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['frames_in_flight'], d.get('depth_tuning_ms'), u.get('ms_per_step'), (d.get('batch_check') or {}).get('last_frame_equal'))"; done
