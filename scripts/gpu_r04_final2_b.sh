#!/bin/bash
# r04 final (second), part B: rocprofv3 kernel trace of the 20-step C3 bench (20 frames per
# launch) and PMC passes; emulated per-rank shards (strong) with multi-frame launches;
# the material bench's kernel trace and PMC passes (profiles/pmc_mat.json).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r04_final2
O=gpurun_out/r04_final2
CONFIG=c3 STEPS=20 bash scripts/gpu_profile.sh || exit $?
for s in "c3 0/2" "c3 1/2" "c3 0/4" "c3 3/4" "c3 0/8" "c3 7/8" "c4 0/8" "c4 7/8"; do
  set -- $s
  timeout -k 10 300 python bench.py --config $1 --emulate-shard $2 --steps 20 --warmup 5 --no-cpu-baseline > $O/shard_${1}_${2/\//of}.log 2>&1
  rc=$?; [ $rc -eq 0 ] || exit $rc
  python3 -c "import json; d=json.loads([l for l in open('$O/shard_${1}_${2/\//of}.log') if l.startswith('{')][-1]); print('shard $1 $2', d['ms_per_step'], d['roofline']['avg_launch_ms'], d.get('frames_per_launch'))"
done
bash scripts/gpu_profile_mat.sh $O/mat || exit $?
