#!/bin/bash
# kernel timeline of a pipelined C3 run for library builds in $LIBS
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out/pt
for v in ${LIBS:-cur}; do
  L=petershirleyraytracer_amd/lib/libpsrt_$v.so; [ "$v" = cur ] && L=petershirleyraytracer_amd/lib/libpsrt.so
  rm -rf gpurun_out/pt/$v
  PSRT_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pt/$v -o run -- python3 bench.py --no-cpu-baseline --steps 10 --warmup 2 --pipeline ${DEPTH:-3} ${BENCH_ARGS} > gpurun_out/pt/$v.log 2>&1 || exit $?
  f=$(find gpurun_out/pt/$v -name "run_kernel_trace.csv" | head -1); cp $f gpurun_out/pt/${v}_trace.csv
  rm -rf gpurun_out/pt/$v
  python3 -c "import json; d=json.loads(open('gpurun_out/pt/$v.log').read().strip().splitlines()[-1]); print('$v', d['ms_per_step'])"
done
