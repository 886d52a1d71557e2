#!/bin/bash
# r04 session AA/AB: where the 7/8 shard's per-batch time goes outside
# psrt_trace (kernel trace beside the bench's host clock marks).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r04ab
mkdir -p $O
export PSRT_BENCH_TIMELINE=1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- python3 bench.py --emulate-shard 7/8 --steps 20 --warmup 5 --no-cpu-baseline > $O/s8.log 2> $O/s8.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt1 -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/c3.log 2> $O/c3.err || exit $?
find $O -name '*.csv' | head -20
