#!/bin/bash
# r03 (session 2): loop-knob sweep (LIBS, scripts/gpu_lib_ab.sh), then the
# diagnostic section clocks and lane-utilisation probes (PSRT_STAMPS)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r03k
O=gpurun_out/r03k
ROUNDS=${ROUNDS:-2} LIBS="${LIBS:-libpsrt.so}" bash scripts/gpu_lib_ab.sh 2>&1 | tee $O/ab.txt || exit 1
PSRT_STAMPS=1 timeout -k 10 300 python -u scripts/dbg_stats.py > $O/stamps.log 2>&1
echo "stamps rc=$?"; grep -h "psrt_sections\|psrt_util" $O/stamps.log | tail -2
