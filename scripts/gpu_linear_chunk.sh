cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for c in c1 c2; do for lc in 1024 512 256 128 64; do
  PSRT_LINEAR_CHUNK=$lc timeout -k 10 120 python bench.py --config $c --no-cpu-baseline --steps 20 --warmup 3 > gpurun_out/lc.log 2>&1 || exit $?
  python3 -c "import json;d=json.loads(open('gpurun_out/lc.log').read().strip().splitlines()[-1]);print('$c',$lc,d['ms_per_step'],d['unpipelined']['ms_per_step'],d['roofline']['avg_launch_ms'])"
done; done
