#!/bin/bash
# r04 session AH: psrt_reduce with 1 / 2 (default) / 3 / 4 sample tiles in
# flight: parity of the default build, then C3 20 steps under a kernel trace,
# two rounds.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r04ah
mkdir -p $O
L=petershirleyraytracer_amd/lib
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_context.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/parity.log 2>&1 || { tail -20 $O/parity.log; exit 1; }
tail -1 $O/parity.log
for r in 1 2; do
  for lib in libpsrt_if1.so libpsrt.so libpsrt_if3.so libpsrt_if4.so; do
    PSRT_LIB=$L/$lib timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt_${lib}_$r -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/c3_${lib}_$r.log 2> $O/c3_${lib}_$r.err || exit $?
    python3 - <<PY
import csv, json
rows = [x for x in csv.DictReader(open("$O/kt_${lib}_$r/run_kernel_trace.csv")) if "psrt_reduce" in x["Kernel_Name"]]
d = max(int(x["End_Timestamp"]) - int(x["Start_Timestamp"]) for x in rows)
b = json.loads([l for l in open("$O/c3_${lib}_$r.log") if l.startswith("{")][-1])
print("$lib", $r, "reduce(20 frames) ms", d / 1e6, "step", b["ms_per_step"], "trace", b["roofline"]["avg_launch_ms"], b["batch_check"]["last_frame_equal"])
PY
  done
done
