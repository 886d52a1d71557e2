#!/bin/bash
# r06 session ZF: the loop's compile-time thresholds re-swept on the kernel
# with the cheaper generator: trials per iteration (PSRT_RNG_FILL / _EXTRA),
# walk batch, refill minimum; parity subset on each variant, then C3 batched,
# two alternating rounds against the product.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06zf
mkdir -p $O
L=petershirleyraytracer_amd/lib
V="f1e2 f3e0 f3e1 f2e2 wb20 wb28 rm12 rm20"
for v in $V; do
  PSRT_LIB=$L/libpsrt_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/pytest_$v.log 2>&1 || { echo "parity $v failed"; tail -20 $O/pytest_$v.log; exit 1; }
done
echo parity ok
for i in 1 2; do
  for v in base $V; do
    lib=$L/libpsrt_$v.so; [ $v = base ] && lib=$L/libpsrt.so
    PSRT_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline > $O/c3_${v}_$i.log 2>&1 || exit 1
  done
done
for f in $O/c3_*.log; do python3 -c "import json; d=json.loads([l for l in open('$f') if l.startswith('{') and '\"metric\"' in l][-1]); print('$f', d['ms_per_step'], d['roofline']['avg_launch_ms'])"; done
