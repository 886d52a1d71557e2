#!/bin/bash
# r04 session O: WRITE_SIZE calibration for 8-B / 2-B record stores
# (scripts/write_calib.hip).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r04o
mkdir -p $O
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_w -o run -- scripts/write_calib > $O/calib.log 2>&1
rc=$?; echo "calib rc=$rc"; cat $O/calib.log | tail -2; [ $rc -eq 0 ] || exit $rc
python3 - <<'PY'
import csv, glob
rows = {}
for f in glob.glob("gpurun_out/r04o/pmc_w/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].split("(")[0]
        rows.setdefault(name, []).append(float(r["Counter_Value"]) * 1024)
n = 96 << 20
known = {"lin16": 16, "lin8": 8, "lin2": 2, "lin10": 10, "void perm10<false>": 10, "void perm10<true>": 10}
for name, v in rows.items():
    key = next((k for k in known if k in name), None)
    b = known.get(key, 0) * n
    print(f"{name:40s} WRITE_SIZE {sum(v)/len(v)/1e9:8.4f} GB  known {b/1e9:8.4f} GB  ratio {sum(v)/len(v)/b if b else 0:6.3f}")
PY
