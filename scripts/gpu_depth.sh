#!/bin/bash
# frames in flight (--pipeline 1/2/3) x library builds, C3 by default
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/var
for r in $(seq 1 ${ROUNDS:-2}); do for v in ${LIBS:-cur}; do for d in ${DEPTHS:-1 2 3}; do
  L=petershirleyraytracer_amd/lib/libpsrt_$v.so; [ "$v" = cur ] && L=petershirleyraytracer_amd/lib/libpsrt.so
  PSRT_LIB=$L timeout -k 10 120 python bench.py --config ${CONFIG:-c3} --no-cpu-baseline --steps ${STEPS:-20} --warmup 3 --pipeline $d ${BENCH_ARGS} > gpurun_out/var/d.log 2>&1 || { tail -5 gpurun_out/var/d.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/var/d.log').read().strip().splitlines()[-1]); print('$v depth $d round $r ms/step', d['ms_per_step'], 'kernel', d['roofline']['avg_launch_ms'])"
done; done; done
