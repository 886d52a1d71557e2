#!/bin/bash
# r05 session G: direction lists keyed by sphere only (tuning dl_cells=0: a
# 3 MB table) against the full lists and none; material bench, batched.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05g
mkdir -p $O
for i in 1 2; do
  timeout -k 10 300 python scripts/bench_materials.py --cpu-rows 1 --tune dl_cells=0 > $O/mat_sph_$i.log 2>&1 || exit $?
  timeout -k 10 300 python scripts/bench_materials.py --cpu-rows 1 --tune no_dirlist=1 > $O/mat_nodl_$i.log 2>&1 || exit $?
  timeout -k 10 300 python scripts/bench_materials.py --cpu-rows 1 > $O/mat_dl_$i.log 2>&1 || exit $?
done
for f in $O/mat_*.log; do python3 -c "import json; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); r=d['roofline']; print('$f', round(d['value'],1), round(d['kernel_ms'],4), r['frac'], r['box_tests_evaluated_per_launch'], r['full_sphere_tests_per_launch'], d.get('unbatched'))"; done
