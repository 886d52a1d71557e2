#!/bin/bash
# r04 session G: section ablation census of psrt_trace (PSRT_ABLATE = 1..8 on
# the pre-clip kernel, base = PSRT_NO_LAYER_CLIP): C3 kernel time (bench, 20
# frames per launch) and PMC VALU / SALU per one-frame dispatch; then the
# layer clip (default build): parity subset and A/B against base.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r04g
mkdir -p $O
L=petershirleyraytracer_amd/lib
for v in _base _a1 _a2 _a3 _a4 _a5 _a6 _a7 _a8; do
  lib=$L/libpsrt$v.so
  PSRT_LIB=$lib timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/c3$v.log 2>&1 || exit $?
  PSRT_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $O/pmc$v -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --pipeline 1 > $O/pmc$v.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "pmc $v rc=$rc"; exit $rc; }
  python3 scripts/pmc_valu.py $O/pmc$v > $O/pmc$v.json
  python3 -c "import json; d=json.loads([l for l in open('$O/c3$v.log') if l.startswith('{')][-1]); p=json.load(open('$O/pmc$v.json')); print('ablate$v', d['roofline']['avg_launch_ms'], round(p['SQ_INSTS_VALU']/1e9,4), round(p['SQ_INSTS_SALU']/1e9,4), round(p['dispatch_ms'],3))"
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_culling.py tests/test_gpu_culling_kat.py tests/test_gpu_context.py -x -q --timeout 300 --timeout-method thread > $O/pytest_clip.log 2>&1
rc=$?; echo "pytest clip rc=$rc"; tail -2 $O/pytest_clip.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for lib in libpsrt.so libpsrt_base.so; do
    PSRT_LIB=$L/$lib timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/clip_${lib}_$r.log 2>&1 || exit $?
    python3 -c "import json; d=json.loads([l for l in open('$O/clip_${lib}_$r.log') if l.startswith('{')][-1]); print('clip $lib $r', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['executed_box_tests_per_launch'], d['roofline']['executed_sphere_tests_per_launch'], d['batch_check']['last_frame_equal'])"
  done
done
# the 1/8 shard's timed launch as a kernel timeline (where a 20-frame step goes)
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/shard8 -o run -- python3 bench.py --emulate-shard 0/8 --steps 20 --warmup 5 --no-cpu-baseline > $O/shard8.log 2>&1 || exit $?
python3 -c "import json; d=json.loads([l for l in open('$O/shard8.log') if l.startswith('{')][-1]); print('shard 0/8', d['ms_per_step'], d['roofline']['avg_launch_ms'])"
