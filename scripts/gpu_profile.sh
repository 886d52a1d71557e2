#!/bin/bash
# rocprofv3 passes over one bench configuration (kernel trace + stats, then
# PMC passes, each on its own). Usage: CONFIG=c3 STEPS=2 bash scripts/gpu_profile.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
CONFIG=${CONFIG:-c3}
STEPS=${STEPS:-2}
OUT=${OUTDIR:-gpurun_out/prof_${CONFIG}}
mkdir -p $OUT
B="bench.py --config $CONFIG --steps $STEPS --warmup 1 --no-cpu-baseline --pipeline 1"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $B > $OUT/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; tail -2 $OUT/trace.log; [ $rc -eq 0 ] || exit $rc
for pmc in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INST_CYCLES_VMEM SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_BRANCH" \
           "SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_IOPS SQ_ACTIVE_INST_VALU2 SQ_INSTS_VMEM"; do
  tag=$(echo $pmc | cut -d' ' -f1)
  timeout -k 10 600 rocprofv3 --pmc $pmc --output-format csv -d $OUT/pmc_$tag -o run -- python3 bench.py --config $CONFIG --steps 1 --warmup 0 --no-cpu-baseline --pipeline 1 > $OUT/pmc_$tag.log 2>&1
  rc=$?; echo "pmc $tag rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
