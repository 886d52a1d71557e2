cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
i=0
for mb in 4096 16384; do for d in 1 2; do
  i=$((i+1))
  PSRT_SAMPLE_BUF_MB=$mb timeout -k 10 200 python bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline --pipeline $d > gpurun_out/c4ab_$i.log 2>&1 || exit $?
  python3 -c "import json; d=json.loads(open('gpurun_out/c4ab_$i.log').read().strip().splitlines()[-1]); print('mb $mb depth $d', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['unpipelined'])"
done; done
