#!/bin/bash
# r06 session F: PMC instruction counts of psrt_trace for the product and the
# trial-gate variants rg1 / rg16 (session E): VALU / SALU instructions, lane
# cycles, one pass each (C3, one frame per dispatch).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06f
mkdir -p $O
L=petershirleyraytracer_amd/lib
for v in base rg1 rg16; do
  lib=$L/libpsrt_$v.so; [ $v = base ] && lib=$L/libpsrt.so
  PSRT_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_$v -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --batch 1 > $O/pmc_$v.log 2>&1 || { tail -5 $O/pmc_$v.log; exit 1; }
  python3 scripts/pmc_valu.py $O/pmc_$v > $O/pmc_$v.json
  cat $O/pmc_$v.json
done
