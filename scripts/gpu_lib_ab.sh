#!/bin/bash
# C3 bench A/B of library builds (LIBS), ROUNDS rounds, interleaved
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-2}); do for lib in ${LIBS:-libpsrt.so}; do
  PSRT_LIB=petershirleyraytracer_amd/lib/$lib timeout -k 10 300 python bench.py --config ${CONFIG:-c3} --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/lab_$lib.$r.log 2>&1 || exit $?
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/lab_$lib.$r.log') if l.startswith('{')][-1]); print('$lib round $r', round(d['value'],1), d['ms_per_step'], 'kernel/frame', d['roofline']['avg_launch_ms'])"
done; done
