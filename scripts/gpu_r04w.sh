#!/bin/bash
# r04 session W: emulated strong shards of C3 and C4 with the new queue
# defaults (k = 2, d = 2), and the C3 / C1 bench lines beside them; then
# 768-thread trace workgroups (two per CU, the same 24 waves) A/B on C3; the
# material walk batch.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r04w
mkdir -p $O
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_c3.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --config c1 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_c1.log 2>&1 || exit $?
for f in $O/bench_c3.log $O/bench_c1.log; do python3 -c "import json; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); print('$f', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"; done
for s in "c3 0/2" "c3 1/2" "c3 0/4" "c3 3/4" "c3 0/8" "c3 7/8" "c4 0/8" "c4 7/8"; do
  set -- $s
  timeout -k 10 300 python bench.py --config $1 --emulate-shard $2 --steps 20 --warmup 5 --no-cpu-baseline > $O/shard_${1}_${2/\//of}.log 2>&1 || exit $?
  python3 -c "import json; d=json.loads([l for l in open('$O/shard_${1}_${2/\//of}.log') if l.startswith('{')][-1]); print('shard $1 $2', d['ms_per_step'], d['roofline']['avg_launch_ms'], d.get('frames_per_launch'))"
done
for r in 1 2 3; do
  for lib in libpsrt.so libpsrt_b768.so; do
    PSRT_LIB=petershirleyraytracer_amd/lib/$lib timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b768_${lib}_$r.log 2>&1 || exit $?
    python3 -c "import json; d=json.loads([l for l in open('$O/b768_${lib}_$r.log') if l.startswith('{')][-1]); print('blk $lib $r', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['batch_check']['last_frame_equal'])"
  done
done
# the material kernel's walk batch under the lens lists (PSRT_MAT_BATCH)
for r in 1 2; do
  for b in 48 32 40 56; do
    PSRT_MAT_BATCH=$b timeout -k 10 300 python scripts/bench_materials.py --spp 10 --cpu-rows 1 > $O/matb_${b}_$r.log 2>&1 || exit $?
    python3 -c "import json; d=json.loads([l for l in open('$O/matb_${b}_$r.log') if l.startswith('{')][-1]); print('matb $b $r', round(d['value'],1), round(d['kernel_ms'],4))"
  done
done
