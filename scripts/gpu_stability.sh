cd "${GRAFT_REPO_ROOT:-/root/repo}"
for r in 1 2 3 4; do
  for v in base w3h2 cur; do
    L=petershirleyraytracer_amd/lib/libpsrt_$v.so; [ $v = cur ] && L=petershirleyraytracer_amd/lib/libpsrt.so
    PSRT_LIB=$L timeout -k 10 120 python bench.py --no-cpu-baseline > gpurun_out/st_$v.log 2>&1 || exit 1
    PSRT_LIB=$L timeout -k 10 120 python bench.py --no-cpu-baseline --config c2 --steps 2 --warmup 1 > gpurun_out/st2_$v.log 2>&1 || exit 1
    python3 -c "import json; d=json.loads(open('gpurun_out/st_$v.log').read().strip().splitlines()[-1]); e=json.loads(open('gpurun_out/st2_$v.log').read().strip().splitlines()[-1]); print('$v', r'$r', 'c3', d['ms_per_step'], d['roofline']['avg_launch_ms'], 'c2(2 steps)', e['ms_per_step'])"
  done
done
