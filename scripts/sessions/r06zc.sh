#!/bin/bash
# r06 session ZC: the final tree's records after the generator change: GPU suite,
# smoke, the default bench line (the driver's command) and two more C3 lines,
# one frame per launch (auto depth), C1, C2, C4, C5, the material bench, and
# the driver's 8-rank command rehearsed on one GPU over gloo for C3 and C4.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06zc
R=gpurun_out/r06zc/rehearsal8
mkdir -p $O $R
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > $O/bench_default.log 2>&1 || exit $?
for i in 2 3; do timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_c3_$i.log 2>&1 || exit $?; done
timeout -k 10 300 python bench.py --no-cpu-baseline --batch 1 > $O/bench_c3_batch1.log 2>&1 || exit $?
for c in c1 c2; do timeout -k 10 300 python bench.py --config $c --cpu-seconds 3 > $O/bench_$c.log 2>&1 || exit $?; done
for c in c4 c5; do timeout -k 10 600 python bench.py --config $c --cpu-seconds 3 > $O/bench_$c.log 2>&1 || exit $?; done
timeout -k 10 300 python scripts/bench_materials.py > $O/mat_batched.log 2>&1 || exit $?
timeout -k 10 300 python scripts/bench_materials.py --batch 1 --cpu-rows 1 > $O/mat_one.log 2>&1 || exit $?
export PSRT_BENCH_BACKEND=gloo MASTER_ADDR=127.0.0.1 OMP_NUM_THREADS=2
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 8 --config c3 > $R/c3_n8.log 2>&1 || { tail -30 $R/c3_n8.log; exit 1; }
grep '^{' $R/c3_n8.log | tail -1 > $R/c3_n8.json
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29542 bench.py --gpus 8 --config c4 --steps 1 --warmup 0 > $R/c4_n8.log 2>&1 || { tail -30 $R/c4_n8.log; exit 1; }
grep '^{' $R/c4_n8.log | tail -1 > $R/c4_n8.json
for f in $O/bench_*.log $O/mat_*.log; do python3 -c "import json; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); r=d['roofline']; u=d.get('unbatched') or {}; print('$f', round(d['value'],1), d['ms_per_step'], r['avg_launch_ms'], r['frac'], d.get('frames_in_flight'), u.get('value'), u.get('ms_per_step'), u.get('frames_in_flight'))"; done
python3 - <<'PY'
import json
for c in ("c3", "c4"):
    d = json.load(open(f"gpurun_out/r06zc/rehearsal8/{c}_n8.json"))
    print(c, d["value"], d["ms_per_step"], len(d["per_rank"]), d["parity_vs_cpu"].get("checked"), d["parity_vs_cpu"].get("ranks_covered"), d["batch_check"].get("all_ranks_equal"), d.get("host_frame_check"))
PY
