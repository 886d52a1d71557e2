#!/bin/bash
# full GPU suite + smoke + default bench + profile of the default bench
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash scripts/gpu_check.sh || exit $?
CONFIG=c3 STEPS=2 bash scripts/gpu_profile.sh
