#!/bin/bash
# Quick A/B: parity subset (fixtures + culling + context), then C3 bench ROUNDS times.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
if [ -z "$NOTEST" ]; then
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_context.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_ab.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_ab.log; [ $rc -eq 0 ] || exit $rc
fi
for r in $(seq 1 ${ROUNDS:-2}); do
  timeout -k 10 300 python bench.py --config ${CONFIG:-c3} --steps 20 --warmup 5 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/ab_$r.log 2>&1 || exit $?
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/ab_$r.log') if l.startswith('{')][-1]); print('round $r value', d['value'], 'ms/step', d['ms_per_step'], 'kernel/frame', d['roofline']['avg_launch_ms'], 'frac', d['roofline']['frac'], 'unbatched', d.get('unbatched'))"
done
