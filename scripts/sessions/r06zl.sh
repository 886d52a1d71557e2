#!/bin/bash
# r06 session ZL: psrt_reduce's tile shape re-measured now that it writes the
# frame's bytes across the link (pinned host memory): tiles of 16 / 32
# samples, 1-3 in flight; C3 batched (20 frames reduced in one launch), the
# reduce's share = step - trace per frame; two alternating rounds.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06zl
mkdir -p $O
L=petershirleyraytracer_amd/lib
V="t16f2 t16f3 t32f1 t32f3"
for v in $V; do
  PSRT_LIB=$L/libpsrt_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/pytest_$v.log 2>&1 || { echo "parity $v failed"; tail -20 $O/pytest_$v.log; exit 1; }
done
echo parity ok
for i in 1 2; do
  for v in base $V; do
    lib=$L/libpsrt_$v.so; [ $v = base ] && lib=$L/libpsrt.so
    PSRT_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline > $O/c3_${v}_$i.log 2>&1 || exit 1
  done
done
for f in $O/c3_*.log; do python3 -c "import json; d=json.loads([l for l in open('$f') if l.startswith('{') and '\"metric\"' in l][-1]); print('$f', d['ms_per_step'], d['roofline']['avg_launch_ms'], round(d['ms_per_step']-d['roofline']['avg_launch_ms'],3))"; done
