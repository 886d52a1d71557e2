#!/bin/bash
# r06 session ZH: psrt_reduce_lean with an empty-launch guard: the
# frames-in-flight and host tests, then C3 one frame per launch and batched.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06zh
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_inflight.py tests/test_gpu_knobs.py tests/test_gpu_host.py tests/test_gpu_bench.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python bench.py --no-cpu-baseline --batch 1 > $O/c3_batch1.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline > $O/c3.log 2>&1 || exit 1
for f in $O/c3*.log; do python3 -c "import json; d=json.loads([l for l in open('$f') if l.startswith('{') and '\"metric\"' in l][-1]); print('$f', d['value'], d['ms_per_step'], d['frames_in_flight'], (d.get('unbatched') or {}).get('value'))"; done
