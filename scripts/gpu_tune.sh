#!/bin/bash
# default bench (depth / tail-priority tuning) on C3 x3, C2, C1, plus the GPU suite
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/tune
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for c in ${CFGS:-c3 c3 c3 c2 c1}; do
  timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/tune/b.log 2>&1 || { tail -5 gpurun_out/tune/b.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/tune/b.log').read().strip().splitlines()[-1]); print('$c', d['ms_per_step'], d['value'], d['frames_in_flight'], d['tail_priority'], d['depth_tuning_ms'], 'unpiped', (d.get('unpipelined') or {}).get('ms_per_step'), 'kernel', d['roofline']['avg_launch_ms'])"
done
