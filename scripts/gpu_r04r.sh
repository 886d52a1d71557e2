#!/bin/bash
# r04 session R: (1) the walk re-bases far origins at the root-box entry
# hit_quick already found (kept per parked lane) instead of recomputing it in
# FP64: parity subset, C3 A/B against libpsrt_head.so; (2) the three r = 1
# spheres as "big" spheres (PSRT_BIG_RATIO=3: tested on every ray with the
# pre-reject, out of the BVH and the grid) against the tall subtree: parity
# subset under the knob, then C3 and material A/B.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r04r
mkdir -p $O
L=petershirleyraytracer_amd/lib
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_culling.py tests/test_gpu_culling_kat.py -x -q --timeout 300 --timeout-method thread > $O/pytest_t0.log 2>&1
rc=$?; echo "pytest t0 rc=$rc"; tail -2 $O/pytest_t0.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for lib in libpsrt.so libpsrt_head.so; do
    PSRT_LIB=$L/$lib timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/t0_${lib}_$r.log 2>&1 || exit $?
    python3 -c "import json; d=json.loads([l for l in open('$O/t0_${lib}_$r.log') if l.startswith('{')][-1]); print('t0 $lib $r', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['batch_check']['last_frame_equal'])"
  done
done
PSRT_BIG_RATIO=3 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_culling.py tests/test_gpu_materials.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in big3 default; do
    if [ $v = big3 ]; then export PSRT_BIG_RATIO=3; else unset PSRT_BIG_RATIO; fi
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/c3_${v}_$r.log 2>&1 || exit $?
    python3 -c "import json; d=json.loads([l for l in open('$O/c3_${v}_$r.log') if l.startswith('{')][-1]); r=d['roofline']; print('c3 $v $r', d['value'], d['ms_per_step'], r['avg_launch_ms'], r['executed_box_tests_per_launch'], r['executed_sphere_tests_per_launch'], d['batch_check']['last_frame_equal'])"
    timeout -k 10 300 python scripts/bench_materials.py --spp 10 --cpu-rows 1 > $O/mat_${v}_$r.log 2>&1 || exit $?
    python3 -c "import json; d=json.loads([l for l in open('$O/mat_${v}_$r.log') if l.startswith('{')][-1]); print('mat $v $r', round(d['value'],1), round(d['kernel_ms'],4), d['roofline']['executed_box_tests_per_launch'])"
  done
done
