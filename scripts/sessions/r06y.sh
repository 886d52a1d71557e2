#!/bin/bash
# r06 session Y: rt_render with the write_color bytes alone (no FP64 sums to
# host: what the reference's main() prints) into page-locked memory, C3 and
# C2, beside the full outputs; the host-path GPU tests.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06y
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_host.py -x -v --timeout 200 --timeout-method thread > $O/pytest_host.log 2>&1 || { tail -30 $O/pytest_host.log; exit 1; }
tail -1 $O/pytest_host.log
for i in 1 2; do
  for a in "--config c3 --out pinned-bytes" "--config c3 --out pinned" "--config c2 --out pinned-bytes"; do
    timeout -k 10 200 python scripts/host_path.py $a 2>/dev/null >> $O/host_path.txt || exit $?
  done
done
cat $O/host_path.txt
