#!/bin/bash
# r06 session J: the launch's units handed out last first (PSRT_REVERSE_UNITS;
# the sky rows last), re-measured on the r06 kernel after the tail model
# (profiles/r06_tailmodel) predicted it would remove the path-length drain:
# parity subset on the variant, then C3 one frame per launch and batched, and
# the emulated 7/8 shard, three alternating rounds.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06j
mkdir -p $O
L=petershirleyraytracer_amd/lib
PSRT_LIB=$L/libpsrt_rev.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_culling_kat.py -x -q --timeout 200 --timeout-method thread > $O/pytest_rev.log 2>&1 || { tail -30 $O/pytest_rev.log; exit 1; }
tail -1 $O/pytest_rev.log
for i in 1 2 3; do
  for v in base rev; do
    lib=$L/libpsrt_$v.so; [ $v = base ] && lib=$L/libpsrt.so
    PSRT_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline > $O/c3_${v}_$i.log 2>&1 || exit 1
    PSRT_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --batch 1 > $O/c3one_${v}_$i.log 2>&1 || exit 1
    PSRT_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --emulate-shard 7/8 > $O/s78_${v}_$i.log 2>&1 || exit 1
  done
done
for f in $O/c3*.log $O/s78*.log; do python3 -c "import json; d=json.loads([l for l in open('$f') if l.startswith('{') and '\"metric\"' in l][-1]); u=d.get('unbatched') or {}; print('$f', d['ms_per_step'], d['roofline']['avg_launch_ms'], u.get('ms_per_step'), u.get('kernel_ms'))"; done
