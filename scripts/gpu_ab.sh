#!/bin/bash
# GPU parity suite, then an A/B of the built library against a baseline build
# (petershirleyraytracer_amd/lib/libpsrt_base.so) on C3 and a 1/8 shard, then
# the diagnostic ray-mix probes of the current build.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
B=petershirleyraytracer_amd/lib/libpsrt_base.so
KNOBS="PSRT_LIB=$B DEFAULT=1 PSRT_LIB=$B DEFAULT=1" SHARDS="${SHARDS:-0/1 0/8}" bash scripts/gpu_knobs.sh || exit $?
PSRT_STAMPS=1 timeout -k 10 120 python bench.py --no-cpu-baseline --steps 1 --warmup 1 > gpurun_out/waves.log 2>&1 || exit $?
grep -E "psrt_util" gpurun_out/waves.log | tail -1
