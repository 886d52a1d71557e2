#!/bin/bash
# r04 session L: section ablation census of the material kernel
# (PSRT_MAT_ABLATE = 1..5): kernel time (book scene 1200x800x10) and PMC
# VALU / SALU instructions per dispatch.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r04l
mkdir -p $O
L=petershirleyraytracer_amd/lib
timeout -k 10 300 python -u -m pytest tests/test_gpu_materials.py -x -q --timeout 200 --timeout-method thread > $O/pytest_mat.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 $O/pytest_mat.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
for v in "" _ma1 _ma2 _ma3 _ma4 _ma5; do
  lib=$L/libpsrt$v.so
  PSRT_LIB=$lib timeout -k 10 300 python scripts/bench_materials.py --spp 10 --cpu-rows 1 > $O/mat${v}_$r.log 2>&1 || exit $?
  if [ $r -eq 1 ]; then
    PSRT_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $O/pmc$v -o run -- python3 scripts/bench_materials.py --spp 10 --cpu-rows 1 --steps 2 --warmup 0 > $O/pmc$v.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "pmc $v rc=$rc"; exit $rc; }
    python3 scripts/pmc_valu.py $O/pmc$v "psrt_trace_mat<true, true, false>" > $O/pmc$v.json
  fi
  python3 -c "import json; d=json.loads([l for l in open('$O/mat${v}_$r.log') if l.startswith('{')][-1]); p=json.load(open('$O/pmc$v.json')); print('ablate$v $r', round(d['kernel_ms'],4), round(p['SQ_INSTS_VALU']/1e9,4), round(p['SQ_INSTS_SALU']/1e9,4), round(p['dispatch_ms'],3))"
done
done
