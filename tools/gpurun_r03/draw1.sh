#!/bin/bash
# Linear-site theta draw: new tests first, then the full GPU suite, then C4/C3 bench lines.
set -u
mkdir -p gpurun_out
run() { local t=$1; shift; local log=$1; shift; timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; return $rc; }
run 300 draw1_new.log python -u -m pytest tests/test_gpu_linear_draw.py -m gpu -v -x --timeout 120 --timeout-method thread -p no:cacheprovider || exit 1
run 900 draw1_tests.log python -u -m pytest tests -m gpu -q --maxfail=5 --timeout 240 --timeout-method thread -p no:cacheprovider || exit 1
for c in c4 c3; do
  run 200 draw1_bench_$c.log python -u bench.py --config $c --no-cpu-baseline --no-other-configs --steps 50 --warmup 5 || exit 1
  MININF_AMD_DRAW_IN_LINEAR=0 run 200 draw1_bench_${c}_off.log python -u bench.py --config $c --no-cpu-baseline --no-other-configs --steps 50 --warmup 5 || exit 1
done
exit 0
