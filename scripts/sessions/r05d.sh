#!/bin/bash
# r05 session D: (1) the material kernel's guided work queue (MatArgs::ph_*):
# the material and context GPU tests, then the material bench batched and one
# frame per launch, twice each; (2) the psrt_trace write-traffic A/B: record
# stores non-temporal (default) or temporal, work chunk 1024 / 512 / 256
# (scripts/build_variants.py libs), a C3 bench line and a WRITE_SIZE pass each.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05d
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_materials.py tests/test_gpu_context.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_mat.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_mat.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python scripts/bench_materials.py --cpu-rows 1 > $O/mat_batched_$i.log 2>&1 || exit $?
  timeout -k 10 300 python scripts/bench_materials.py --batch 1 --cpu-rows 1 > $O/mat_one_$i.log 2>&1 || exit $?
done
L=petershirleyraytracer_amd/lib
for i in 1 2; do
  for v in "" _tstore _tstore512 _tstore256 _nt256; do
    PSRT_LIB=$L/libpsrt$v.so timeout -k 10 300 python bench.py --no-cpu-baseline > $O/wab${v:-_base}_$i.log 2>&1 || exit $?
  done
done
for v in "" _tstore _tstore512 _tstore256 _nt256; do
  PSRT_LIB=$L/libpsrt$v.so timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/wpmc${v:-_base} -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --pipeline 1 > $O/wpmc${v:-_base}.log 2>&1 || exit $?
  echo "pmc $v done"
done
for f in $O/mat_*.log $O/wab_*.log; do python3 -c "import json; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); r=d['roofline']; print('$f', round(d['value'],1), round(d['ms_per_step'],4), r['avg_launch_ms'], r['frac'], d.get('unbatched'))"; done
