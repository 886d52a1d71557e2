#!/bin/bash
# r05 session I: direction lists capped at 3 / 2 entries (a wave runs its
# longest lane's list), full and sphere-keyed, against none; material bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05i
mkdir -p $O
L=petershirleyraytracer_amd/lib
for i in 1 2; do
  for v in cap3 cap2; do
    PSRT_LIB=$L/libpsrt_$v.so timeout -k 10 300 python scripts/bench_materials.py --cpu-rows 1 > $O/mat_${v}_dl_$i.log 2>&1 || exit $?
    PSRT_LIB=$L/libpsrt_$v.so timeout -k 10 300 python scripts/bench_materials.py --cpu-rows 1 --tune dl_cells=0 > $O/mat_${v}_sph_$i.log 2>&1 || exit $?
  done
  timeout -k 10 300 python scripts/bench_materials.py --cpu-rows 1 --tune no_dirlist=1 > $O/mat_nodl_$i.log 2>&1 || exit $?
done
for f in $O/mat_*.log; do python3 -c "import json; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); r=d['roofline']; print('$f', round(d['value'],1), round(d['kernel_ms'],4), r['frac'], r['box_tests_evaluated_per_launch'], r['full_sphere_tests_per_launch'])"; done
