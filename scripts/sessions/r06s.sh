#!/bin/bash
# r06 session S: frames in flight in the bench (the auto depth now tunes over
# 10+ frames with a 1% bar; a batched line's `unbatched` rate tries two in
# flight); the lean reduce's issue priority 0 / 1 / 3 (A/B builds); the 7/8
# C3 shard as 2 launches of 10 frames in flight against one of 20.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06s
mkdir -p $O
L=petershirleyraytracer_amd/lib
timeout -k 10 500 python -u -m pytest tests/test_gpu_inflight.py tests/test_gpu_bench.py -k "inflight or frames_in_flight or lean or single_gpu" -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2 3; do
  for v in prio0 prio1 prio3; do
    lib=$L/libpsrt_$v.so; [ $v = prio3 ] && lib=$L/libpsrt.so
    PSRT_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --batch 1 --pipeline 2 > $O/c3p2_${v}_$i.log 2>&1 || exit 1
  done
  timeout -k 10 200 python bench.py --no-cpu-baseline --emulate-shard 7/8 > $O/s78_b20_$i.log 2>&1 || exit 1
  timeout -k 10 200 python bench.py --no-cpu-baseline --emulate-shard 7/8 --batch 10 --pipeline 2 > $O/s78_b10p2_$i.log 2>&1 || exit 1
done
timeout -k 10 200 python bench.py --no-cpu-baseline --batch 1 > $O/c3auto.log 2>&1 || exit 1
timeout -k 10 300 python bench.py > $O/c3default.log 2>&1 || exit 1
for f in $O/c3*.log $O/s78*.log; do python3 -c "import json; d=json.loads([l for l in open('$f') if l.startswith('{') and '\"metric\"' in l][-1]); u=d.get('unbatched') or {}; print('$f', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['frames_in_flight'], d.get('depth_tuning_ms'), u)"; done
