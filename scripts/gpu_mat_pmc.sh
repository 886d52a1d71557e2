#!/bin/bash
# PMC passes over the material bench (one pass per counter group)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/prof_mat_pmc
mkdir -p $O
for pmc in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64" "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_CVT SQ_WAIT_INST_LDS SQ_INSTS_SMEM"; do
  tag=$(echo $pmc | cut -d' ' -f1)
  timeout -k 10 300 rocprofv3 --pmc $pmc --output-format csv -d $O/pmc_$tag -o run -- python3 scripts/bench_materials.py --spp 10 --steps 2 --warmup 0 --cpu-rows 1 > $O/pmc_$tag.log 2>&1
  rc=$?; echo "pmc $tag rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
