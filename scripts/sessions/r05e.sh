#!/bin/bash
# r05 session E: the rocprofv3 records of the product build: C3 kernel trace +
# stats (20 frames per launch, as the bench line) and the PMC passes; the
# material bench's trace and PMC passes (one frame per dispatch).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05e
mkdir -p $O
OUTDIR=$O/prof_c3 CONFIG=c3 STEPS=20 bash scripts/gpu_profile.sh || exit $?
OUTDIR=$O/prof_mat bash scripts/gpu_profile_mat.sh $O/prof_mat_sum || exit $?
