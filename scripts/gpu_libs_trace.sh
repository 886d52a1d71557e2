#!/bin/bash
# Kernel-trace stats of bench.py (C3) for several library builds:
# LIBS="default petershirleyraytracer_amd/lib/libpsrt_x.so ..." bash scripts/gpu_libs_trace.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/libs
i=0
for L in ${LIBS:-default}; do
  i=$((i+1))
  E=""; [ "$L" != "default" ] && E="PSRT_LIB=$L"
  env $E timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/libs/t$i -o run -- python3 bench.py --no-cpu-baseline --steps ${STEPS:-5} --warmup 1 ${BENCH_ARGS} > gpurun_out/libs/t$i.log 2>&1 || exit $?
  echo "== $L: $(python3 -c "import json; d=json.loads(open('gpurun_out/libs/t$i.log').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['roofline']['avg_launch_ms'])")"
  cut -d, -f1-4 gpurun_out/libs/t$i/run_kernel_stats.csv | grep -v fillBuffer | cut -c1-40,150-
done
