#!/bin/bash
# C4 / C5 on one GPU with the default 16 GiB sample buffer against larger caps
# (fewer sample chunks, so fewer launch tails per frame).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for cfg in "c4 2 1" "c5 2 1"; do
  set -- $cfg
  for mb in 16384 49152 98304; do
    PSRT_SAMPLE_BUF_MB=$mb timeout -k 10 300 python bench.py --config $1 --steps $2 --warmup $3 --no-cpu-baseline > gpurun_out/buf_$1_$mb.log 2>&1
    rc=$?; echo "$1 buf=$mb rc=$rc $(tail -1 gpurun_out/buf_$1_$mb.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])' 2>&1)"
    [ $rc -eq 0 ] || exit $rc
  done
done
