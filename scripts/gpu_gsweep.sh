cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for G in 2 4 8 16 32 64 128 1200; do
  timeout -k 10 120 python bench.py --steps 10 --warmup 2 --emulate-shard 0/$G > gpurun_out/g_$G.log 2>&1 || exit $?
  python3 -c "import json; d=json.loads(open('gpurun_out/g_$G.log').read().strip().splitlines()[-1]); print('G=$G', d['ms_per_step'], d['roofline']['avg_launch_ms'], d['rays_per_sample'])"
done
for G in 8 64; do
  PSRT_STAMPS=1 timeout -k 10 120 python bench.py --steps 2 --warmup 1 --emulate-shard 0/$G > gpurun_out/gs_$G.log 2>&1 || exit $?
  grep -E "psrt_" gpurun_out/gs_$G.log | tail -3
done
