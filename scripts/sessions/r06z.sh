#!/bin/bash
# r06 session Z: bytes-only host frames (psrt::basic_frame::want_accum, the
# CLI without --accum): the host API tests, the CLI end to end on C3 (md5),
# and rt_render into page-locked bytes alone.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06z
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_host_api.py tests/test_gpu_host.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
  ( time timeout -k 10 120 petershirleyraytracer_amd/bin/raytracer --scene final --width 1200 --height 800 --spp 100 -o $O/cli_c3.ppm ) > $O/cli_c3_$i.txt 2>&1 || exit $?
  md5sum $O/cli_c3.ppm >> $O/cli_c3_$i.txt && rm -f $O/cli_c3.ppm
done
cat $O/cli_c3_2.txt
timeout -k 10 200 python scripts/host_path.py --config c3 --out pinned-bytes 2>/dev/null > $O/host_path.txt || exit $?
cat $O/host_path.txt
