#!/bin/bash
# r06 session Q: co-residency probe: do 64-thread workgroups of another
# stream get CU slots while a C3 psrt_trace launch fills the GPU?
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06q
mkdir -p $O
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -shared -o $O/probe.so scripts/coresident_probe.hip || exit 1
timeout -k 10 120 python scripts/coresident_probe.py $O/probe.so > $O/probe.txt 2>&1; rc=$?
cat $O/probe.txt; exit $rc
