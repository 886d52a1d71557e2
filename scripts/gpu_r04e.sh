#!/bin/bash
# r04 session E: section census of the current psrt_trace (diagnostic stamps
# build: section clocks only, util probes compiled out), C3 one frame.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r04e
mkdir -p $O
PSRT_LIB=petershirleyraytracer_amd/lib/libpsrt_nutil.so timeout -k 10 300 python scripts/stamps_c3.py > $O/stamps_nutil.log 2>&1 || exit $?
tail -3 $O/stamps_nutil.log
timeout -k 10 300 python scripts/stamps_c3.py > $O/stamps_util.log 2>&1 || exit $?
tail -3 $O/stamps_util.log
