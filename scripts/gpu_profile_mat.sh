#!/bin/bash
# rocprofv3 passes over the material bench (kernel trace + stats, then PMC
# passes, each on its own), summarised into profiles/pmc_mat.json by
# scripts/summarize_profile.py. Usage: bash scripts/gpu_profile_mat.sh <dst>
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
DST=${1:-profiles/mat}
OUT=${OUTDIR:-gpurun_out/prof_mat}
mkdir -p $OUT
B="scripts/bench_materials.py --spp 10 --cpu-rows 1 --batch 1"  # one frame per dispatch
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $B > $OUT/trace.log 2>&1
rc=$?; echo "mat trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
for pmc in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_INSTS_SMEM"; do
  tag=$(echo $pmc | cut -d' ' -f1)
  timeout -k 10 300 rocprofv3 --pmc $pmc --output-format csv -d $OUT/pmc_$tag -o run -- python3 $B --steps 2 --warmup 0 > $OUT/pmc_$tag.log 2>&1
  rc=$?; echo "mat pmc $tag rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
PSRT_TIMED_KERNEL="psrt_trace_mat<true, true, false>" python3 scripts/summarize_profile.py $OUT $DST mat
