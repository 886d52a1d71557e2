#!/bin/bash
# r05 session N: psrt_reduce_rgb with LDS-staged tiles: the material GPU tests
# (chunked, multi-frame, shards), the material bench (batched, one frame per
# launch) and its kernel trace.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05n
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_materials.py tests/test_gpu_sweep.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python scripts/bench_materials.py --cpu-rows 1 > $O/mat_batched_$i.log 2>&1 || exit $?
  timeout -k 10 300 python scripts/bench_materials.py --cpu-rows 1 --batch 1 > $O/mat_one_$i.log 2>&1 || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 scripts/bench_materials.py --cpu-rows 1 --batch 1 > $O/trace.log 2>&1 || exit $?
grep -h "psrt_reduce_rgb\|psrt_trace_mat<true, true, false>" $O/trace/*kernel_stats.csv | cut -c1-160
for f in $O/mat_*.log; do python3 -c "import json; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); print('$f', round(d['value'],1), round(d['ms_per_step'],4), round(d['kernel_ms'],4))"; done
