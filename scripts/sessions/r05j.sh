#!/bin/bash
# r05 session J: the product build's records: GPU suite, smoke, the default
# bench line, the C3 rocprofv3 trace (20 frames per launch, as the bench) and
# PMC passes, the material bench's trace and PMC passes.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05j
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > $O/bench_default.log 2>&1 || exit $?
OUTDIR=$O/prof_c3 CONFIG=c3 STEPS=20 bash scripts/gpu_profile.sh || exit $?
OUTDIR=$O/prof_mat bash scripts/gpu_profile_mat.sh $O/prof_mat_sum || exit $?
