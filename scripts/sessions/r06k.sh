#!/bin/bash
# r06 session K: kernel timelines of one-frame-per-launch C3 with 1 and 2
# frames in flight (where does the second frame's trace start, what fills the
# first one's tail)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06k
mkdir -p $O
for d in 1 2; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/p$d -o run -- python3 bench.py --batch 1 --pipeline $d --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_p$d.log 2>&1 || exit $?
done
find $O -name "*kernel_trace.csv" | head
