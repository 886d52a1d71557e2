#!/bin/bash
# r06 session M: session L again after the drain flag went to one workgroup in
# 64 (12k same-word stores per launch cost ~1 ms): timeline of 3 in flight
# (gated), parity subset, the flag A/B and 1 / 2 / 3 in flight.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06m
mkdir -p $O
L=petershirleyraytracer_amd/lib
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/p3g -o run -- python3 bench.py --batch 1 --pipeline 3 --steps 10 --warmup 2 --no-cpu-baseline > $O/trace_p3g.log 2>&1 || { tail -20 $O/trace_p3g.log; exit 1; }
grep '^{' $O/trace_p3g.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('p3 gated', d['ms_per_step'], d['frames_in_flight'])"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_culling_kat.py -x -q --timeout 200 --timeout-method thread > $O/pytest_sub.log 2>&1 || { tail -30 $O/pytest_sub.log; exit 1; }
tail -1 $O/pytest_sub.log
for i in 1 2 3; do
  for v in noflag flag; do
    lib=$L/libpsrt_$v.so; [ $v = flag ] && lib=$L/libpsrt.so
    PSRT_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline > $O/c3_${v}_$i.log 2>&1 || exit 1
    PSRT_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --batch 1 --pipeline 1 > $O/c3one_${v}_$i.log 2>&1 || exit 1
  done
  for d in 2 3; do
    timeout -k 10 200 python bench.py --no-cpu-baseline --batch 1 --pipeline $d > $O/c3p${d}g_$i.log 2>&1 || exit 1
  done
  timeout -k 10 200 python bench.py --no-cpu-baseline --batch 1 --pipeline 2 --no-drain-gate > $O/c3p2n_$i.log 2>&1 || exit 1
done
timeout -k 10 200 python bench.py --no-cpu-baseline --batch 1 > $O/c3auto.log 2>&1 || exit 1
for f in $O/c3*.log; do python3 -c "import json; d=json.loads([l for l in open('$f') if l.startswith('{') and '\"metric\"' in l][-1]); u=d.get('unbatched') or {}; print('$f', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['frames_in_flight'], d.get('depth_tuning_ms'), u.get('ms_per_step'))"; done
