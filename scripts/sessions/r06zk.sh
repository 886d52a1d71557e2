#!/bin/bash
# r06 session ZK: the material kernel's PMC passes again (its counter stream's
# generator changed with r06's contract; the kernel code is unchanged since
# r05), then the material bench lines that read the refreshed summary.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06zk
mkdir -p $O
OUTDIR=$O/prof_mat bash scripts/gpu_profile_mat.sh $O/mat_sum || exit $?
