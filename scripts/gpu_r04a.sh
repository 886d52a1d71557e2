#!/bin/bash
# r04 session A: the GPU suite (bench self-checks, ADVICE fixes), smoke, the
# material kernel's FP32 trial A/B, a C3 bench line, and a PC-sampling probe.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r04a
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for lib in libpsrt.so libpsrt_matf64.so; do
    PSRT_LIB=petershirleyraytracer_amd/lib/$lib timeout -k 10 300 python scripts/bench_materials.py --spp 10 --cpu-rows 1 > $O/mat_${lib}_$r.log 2>&1 || exit $?
    python3 -c "import json; d=json.loads([l for l in open('$O/mat_${lib}_$r.log') if l.startswith('{')][-1]); print('mat $lib $r', round(d['value'],1), round(d['kernel_ms'],4))"
  done
done
timeout -k 10 300 python bench.py > $O/bench_c3.log 2>&1 || exit $?
python3 -c "import json; d=json.loads([l for l in open('$O/bench_c3.log') if l.startswith('{')][-1]); print('c3', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['batch_check'], d['parity_vs_cpu'])"
timeout -k 10 60 rocprofv3 -L > $O/rocprof_list.txt 2>&1; echo "list rc=$?"
grep -i -A12 'pc.sampl' $O/rocprof_list.txt | head -40 || true
