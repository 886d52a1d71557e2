#!/bin/bash
# r04 session AE: wave timelines (PSRT_STAMPS) of the 7/8 and full C3 launch,
# 1 and 20 frames.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r04ae
mkdir -p $O
timeout -k 10 300 python3 scripts/stamps_shard.py 7 8 > $O/s8.txt 2>&1 || exit $?
timeout -k 10 300 python3 scripts/stamps_shard.py 0 1 > $O/c3.txt 2>&1 || exit $?
grep -h "frames\|psrt_waves" $O/s8.txt $O/c3.txt
