#!/bin/bash
# r06 session E: look-ahead trial rounds gated by the lanes that have room
# (PSRT_RNG_GATE; G0 / G1 = lanes needed for round 1 / 2; the extra round for a
# scattering lane without a trial unchanged). Parity subset on two variants,
# then C3 bench A/B, three alternating rounds.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06e
mkdir -p $O
L=petershirleyraytracer_amd/lib
for v in rg16 rg824; do
  PSRT_LIB=$L/libpsrt_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_culling_kat.py tests/test_gpu_sweep.py -x -q --timeout 200 --timeout-method thread > $O/pytest_$v.log 2>&1 || { tail -30 $O/pytest_$v.log; exit 1; }
  tail -1 $O/pytest_$v.log
done
for i in 1 2 3; do
  for v in base rg1 rg16 rg32 rg824 rg48; do
    lib=$L/libpsrt_$v.so; [ $v = base ] && lib=$L/libpsrt.so
    PSRT_LIB=$lib timeout -k 10 200 python bench.py --cpu-seconds 1 > $O/c3_${v}_$i.log 2>&1 || { tail -20 $O/c3_${v}_$i.log; exit 1; }
  done
done
python3 - <<'PY'
import json, glob, os, collections
res = collections.defaultdict(list)
for f in sorted(glob.glob("gpurun_out/r06e/c3_*.log")):
    ls = [l for l in open(f) if l.startswith("{") and '"metric"' in l]
    d = json.loads(ls[-1]); ub = d.get("unbatched") or {}
    v = os.path.basename(f)[3:].rsplit("_", 1)[0]
    res[v].append((d["ms_per_step"], d["roofline"]["achieved"] and round(d.get("kernel_ms_per_frame", 0) or 0, 3), ub.get("ms_per_step")))
for v, r in res.items(): print(v, r)
PY
