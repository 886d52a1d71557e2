#!/bin/bash
# r06 session C: the host-buffer paths before any change:
# D2H options for a C3 frame's outputs (scripts/host_copy_probe.cpp), and
# rt_render / rt_render_devices (1 and 8 members on the one device) for C3 and
# a C4 row band (1/8 of the rows).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06c
mkdir -p $O
timeout -k 10 120 ./scripts/host_copy_probe > $O/probe.json 2>&1 || { cat $O/probe.json; exit 1; }
cat $O/probe.json
for a in "--config c3" "--config c3 --group 1" "--config c3 --group 8" "--config c4 --rows 0/8 --frames 3" "--config c4 --rows 0/8 --frames 3 --group 8"; do
  timeout -k 10 200 python scripts/host_path.py $a >> $O/host_path.txt 2>&1 || { tail -20 $O/host_path.txt; exit 1; }
done
cat $O/host_path.txt
