#!/bin/bash
# r06 session ZD: the final tree's profiles after the generator change: the C3
# rocprofv3 kernel trace + stats (20 frames per launch, as the bench line) and
# PMC passes; the emulated strong-scaling ranks of C3 (every rank of G = 2, 4,
# 8) and C4 (ranks 0 and 7 of 8); the CLI end to end; the host-buffer path;
# a kernel trace of one-frame launches two in flight; rt_render bytes only.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06zd
mkdir -p $O
OUTDIR=$O/prof_c3 CONFIG=c3 STEPS=20 bash scripts/gpu_profile.sh || exit $?
for G in 2 4 8; do
  for ((R=0; R<G; R++)); do
    timeout -k 10 300 python bench.py --no-cpu-baseline --emulate-shard $R/$G > $O/shard_c3_${R}_of_${G}.log 2>&1 || exit $?
  done
done
for R in 0 7; do
  timeout -k 10 600 python bench.py --no-cpu-baseline --config c4 --emulate-shard $R/8 > $O/shard_c4_${R}_of_8.log 2>&1 || exit $?
done
( time timeout -k 10 120 petershirleyraytracer_amd/bin/raytracer --scene final --width 1200 --height 800 --spp 100 -o $O/cli_c3.ppm ) > $O/cli_c3.txt 2>&1 || exit $?
md5sum $O/cli_c3.ppm >> $O/cli_c3.txt && rm -f $O/cli_c3.ppm
for a in "--config c3 --out pinned" "--config c2 --out pinned" "--config c3 --out new" "--config c3 --out pinned-bytes" "--config c2 --out pinned-bytes"; do
  timeout -k 10 200 python scripts/host_path.py $a 2>/dev/null >> $O/host_path.txt || exit $?
done
for f in $O/shard_*.log; do python3 -c "import json; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); print('$f', d['ms_per_step'], d['roofline']['avg_launch_ms'])"; done
cat $O/cli_c3.txt $O/host_path.txt
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/inflight -o run -- python3 bench.py --batch 1 --pipeline 2 --steps 20 --warmup 2 --no-cpu-baseline > $O/inflight.log 2>&1 || exit $?
