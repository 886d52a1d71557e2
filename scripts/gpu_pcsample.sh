#!/bin/bash
# PC sampling of psrt_trace (dynamic per-instruction hot spots):
#   METHOD=stochastic|host_trap bash scripts/gpu_pcsample.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
M=${METHOD:-stochastic}
U=${UNIT:-cycles}
I=${INTERVAL:-1048576}
OUT=gpurun_out/pcs_$M
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 ${PCS_TIMEOUT:-180} rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method $M \
  --pc-sampling-unit $U --pc-sampling-interval $I --output-format csv -d $OUT -o run -- \
  python3 bench.py --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline --pipeline 1 > $OUT/run.log 2>&1
rc=$?; echo "pcs rc=$rc"; tail -3 $OUT/run.log
find $OUT -name "*.csv" | head; exit $rc
