#!/bin/bash
# Knob sweep of psrt_trace under multi-frame launches (C3, 20 frames per launch):
# one bench per setting, kernel ms per frame. Settings are env knobs read by
# psrt_capi.hip (tuning only; defaults unchanged).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --config c3 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/knob_$tag.log 2>&1 || return $?
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/knob_$tag.log') if l.startswith('{')][-1]); print('$tag', '$*', 'value', round(d['value'],1), 'ms/step', d['ms_per_step'], 'kernel/frame', d['roofline']['avg_launch_ms'])"
}
run base A=0 || exit $?
for kv in ${KNOBS:-PSRT_REFILL_MIN=12 PSRT_REFILL_MIN=20 PSRT_BATCH=20 PSRT_BATCH=28 PSRT_WALK_TAIL=2 PSRT_WALK_TAIL=6 PSRT_RNG_EXTRA=0 PSRT_RNG_EXTRA=2 PSRT_QUEUE_D=8 PSRT_QUEUE_K=1}; do
  run "$(echo $kv | tr '=' '_')" "$kv" || exit $?
done
run base2 A=0
