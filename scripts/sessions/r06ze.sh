#!/bin/bash
# r06 session ZE: the bench lines again with the new generator's PMC summary
# (profiles/pmc_c3.json from session ZD) in place: the default line (the
# driver's command, with the CPU baseline), two more C3 lines and one frame
# per launch.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06ze
mkdir -p $O
timeout -k 10 600 python bench.py > $O/bench_default.log 2>&1 || exit $?
for i in 2 3; do timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_c3_$i.log 2>&1 || exit $?; done
timeout -k 10 300 python bench.py --no-cpu-baseline --batch 1 > $O/bench_c3_batch1.log 2>&1 || exit $?
for f in $O/bench_*.log; do python3 -c "import json; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); r=d['roofline']; v=r['valu_issue']; u=d.get('unbatched') or {}; print('$f', round(d['value'],1), d['ms_per_step'], r['avg_launch_ms'], r['frac'], r['traffic'], round(v['insts_per_launch']/1e9,3), round(v['salu_insts_per_launch']/1e9,3), v['lane_utilisation'], v['simd_cycles_per_valu_inst'], d.get('frames_in_flight'), u.get('value'), u.get('ms_per_step'), (d.get('cpu_baseline') or {}).get('value'), (d.get('parity_vs_cpu') or {}).get('fp64_bit_identical'))"; done
