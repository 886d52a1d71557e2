#!/bin/bash
# r04 session J: session I (strided single psrt_reduce launch: parity +
# context + bench tests, A/B against per-frame launches on C3 and the 1/8
# shard), the material kernel's LDS / occupancy / refill variants, and the
# trial-round knobs.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r04j
mkdir -p $O
L=petershirleyraytracer_amd/lib
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_context.py tests/test_gpu_bench.py tests/test_gpu_materials.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for lib in libpsrt_mlean1.so libpsrt_mlean1w6.so libpsrt_mlean2b320.so; do
  PSRT_LIB=$L/$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_materials.py -x -q --timeout 200 --timeout-method thread > $O/pytest_$lib.log 2>&1 || { echo "pytest $lib failed"; tail -5 $O/pytest_$lib.log; exit 1; }
done
echo "mat variant parity ok"
for r in 1 2; do
  for lib in libpsrt.so libpsrt_prevred.so; do
    PSRT_LIB=$L/$lib timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/c3_${lib}_$r.log 2>&1 || exit $?
    PSRT_LIB=$L/$lib timeout -k 10 300 python bench.py --emulate-shard 0/8 --steps 20 --warmup 5 > $O/s8_${lib}_$r.log 2>&1 || exit $?
    python3 -c "
import json
for f in ['$O/c3_${lib}_$r.log','$O/s8_${lib}_$r.log']:
    d=json.loads([l for l in open(f) if l.startswith('{')][-1]); print(f.split('/')[-1], d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
  done
done
for r in 1 2; do
  for lib in libpsrt.so libpsrt_mlean1.so libpsrt_mlean1w6.so libpsrt_mlean2b320.so libpsrt_mref16.so libpsrt_mref8.so; do
    PSRT_LIB=$L/$lib timeout -k 10 300 python scripts/bench_materials.py --spp 10 --cpu-rows 1 > $O/mat_${lib}_$r.log 2>&1 || exit $?
    python3 -c "import json; d=json.loads([l for l in open('$O/mat_${lib}_$r.log') if l.startswith('{')][-1]); print('mat $lib $r', round(d['value'],1), round(d['kernel_ms'],4), d['roofline']['executed_box_tests_per_launch'])"
  done
done
for lib in libpsrt_f2e0.so libpsrt_f3e0.so libpsrt_f1e1.so libpsrt_f1e2.so; do
  PSRT_LIB=$L/$lib timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/rng_${lib}.log 2>&1 || exit $?
  python3 -c "import json; d=json.loads([l for l in open('$O/rng_${lib}.log') if l.startswith('{')][-1]); print('rng $lib', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['batch_check']['last_frame_equal'])"
done
