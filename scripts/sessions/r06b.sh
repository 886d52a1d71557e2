#!/bin/bash
# r06 session B: launch-tail path migration. The GPU suite
# on the migration build, then C3 A/B: base (HEAD kernel, lib/libpsrt_base.so),
# mig (product build, mig_below 16), mig0 (product build, migration off at run
# time), split (the exchange only in a second loop copy); three alternating
# rounds of the default bench (20-frame launch + the one-frame `unbatched`
# rate), then the 7/8 and 0/8 emulated shards.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06b
mkdir -p $O
L=petershirleyraytracer_amd/lib
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
run() {  # name lib extra-args...
  local n=$1 lib=$2; shift 2
  PSRT_LIB=$L/$lib timeout -k 10 200 python bench.py --cpu-seconds 1 "$@" > $O/$n.log 2>&1 || { tail -20 $O/$n.log; exit 1; }
}
for i in 1 2 3; do
  run c3_base_$i libpsrt_base.so
  run c3_mig_$i libpsrt.so
  run c3_mig0_$i libpsrt.so --tune mig_below=0
  run c3_split_$i libpsrt_split.so
  run c3one_base_$i libpsrt_base.so --batch 1 --no-cpu-baseline
  run c3one_mig_$i libpsrt.so --batch 1 --no-cpu-baseline
done
for i in 1 2; do
  for v in base mig; do
    lib=libpsrt.so; [ $v = base ] && lib=libpsrt_base.so
    run s78_${v}_$i $lib --emulate-shard 7/8 --no-cpu-baseline
    run s08_${v}_$i $lib --emulate-shard 0/8 --no-cpu-baseline
  done
done
python3 - <<'PY'
import json, glob, os
rows = {}
for f in sorted(glob.glob("gpurun_out/r06b/*.log")):
    if "pytest" in f: continue
    ls = [l for l in open(f) if l.startswith("{") and '"metric"' in l]
    if not ls: print(f, "no line"); continue
    d = json.loads(ls[-1])
    ub = d.get("unbatched") or {}
    print(os.path.basename(f), round(d["value"], 1), d["ms_per_step"], "unbatched", ub.get("value"), ub.get("ms_per_step"), ub.get("kernel_ms"))
PY
