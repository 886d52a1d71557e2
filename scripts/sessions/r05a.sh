#!/bin/bash
# r05 session A: the GPU suite (new: device groups, far camera, material fault
# hook, overlapping frame buffers), smoke, the default bench line (new roofline
# accounting), and the C3 rocprofv3 trace + PMC passes (with SQ_THREAD_CYCLES_VALU).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05a
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > $O/bench_default.log 2>&1 || exit $?
OUTDIR=$O/prof_c3 CONFIG=c3 STEPS=2 bash scripts/gpu_profile.sh || exit $?
