#!/bin/bash
# Per-rank step time of the multi-GPU bench, emulated on one GPU: strong
# scaling (the C3 frame split over G ranks) and weak scaling (G x spp).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/shards
for sc in strong weak; do
  for sh in 0/1 0/2 1/2 0/4 3/4 0/8 7/8; do
    tag=${sc}_$(echo $sh | tr / _)
    E="--emulate-shard $sh"; [ $sh = 0/1 ] && E="--no-cpu-baseline"
    timeout -k 10 120 python bench.py --steps 20 --warmup 3 --scaling $sc $E > gpurun_out/shards/$tag.log 2>&1 || exit $?
    python3 -c "import json; d=json.loads(open('gpurun_out/shards/$tag.log').read().strip().splitlines()[-1]); print('$sc $sh', d['value'], d['ms_per_step'], d['frames_in_flight'], d.get('depth_tuning_ms'))"
  done
done
