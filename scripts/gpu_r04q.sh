#!/bin/bash
# r04 session Q: walks start below the root (BvhView::walk0: the root box is
# never tested): parity subset, then C3 and material A/B against the previous
# build (libpsrt_head.so).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r04q
mkdir -p $O
L=petershirleyraytracer_amd/lib
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_culling.py tests/test_gpu_culling_kat.py tests/test_gpu_materials.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for lib in libpsrt.so libpsrt_head.so; do
    PSRT_LIB=$L/$lib timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/c3_${lib}_$r.log 2>&1 || exit $?
    python3 -c "import json; d=json.loads([l for l in open('$O/c3_${lib}_$r.log') if l.startswith('{')][-1]); print('c3 $lib $r', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['batch_check']['last_frame_equal'])"
  done
done
for r in 1 2; do
  for lib in libpsrt.so libpsrt_head.so; do
    PSRT_LIB=$L/$lib timeout -k 10 300 python scripts/bench_materials.py --spp 10 --cpu-rows 1 > $O/mat_${lib}_$r.log 2>&1 || exit $?
    python3 -c "import json; d=json.loads([l for l in open('$O/mat_${lib}_$r.log') if l.startswith('{')][-1]); print('mat $lib $r', round(d['value'],1), round(d['kernel_ms'],4), d['roofline']['executed_box_tests_per_launch'])"
  done
done
