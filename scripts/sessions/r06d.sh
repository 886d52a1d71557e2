#!/bin/bash
# r06 session D: page-locked frame outputs (rt_host_alloc, ABI 6; VERDICT r05
# item 4): their GPU tests, then the host-buffer rates of rt_render and the
# device group (C3; a C4 row band) with new / reused pageable / pinned outputs.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06d
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_host.py tests/test_host_api.py tests/test_gpu_group.py tests/test_abi.py tests/test_gpu_knobs.py -m "gpu or not gpu" -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for a in "--out new" "--out reuse" "--out pinned" "--group 1 --out pinned" "--group 8 --out new" "--group 8 --out pinned" "--config c4 --rows 0/8 --frames 3 --out new" "--config c4 --rows 0/8 --frames 3 --out pinned" "--config c4 --rows 0/8 --frames 3 --group 8 --out pinned"; do
  timeout -k 10 200 python scripts/host_path.py $a 2>/dev/null >> $O/host_path.txt || { tail -20 $O/host_path.txt; exit 1; }
done
cat $O/host_path.txt
