#!/bin/bash
# Normal tail of the final gradients: new tests, full suite, C4/C3 bench A/B.
set -u
mkdir -p gpurun_out
run() { local t=$1; shift; local log=$1; shift; timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; return $rc; }
run 300 final2_new.log python -u -m pytest tests/test_gpu_final_grads.py tests/test_gpu_linear_draw.py -m gpu -v -x --timeout 120 --timeout-method thread -p no:cacheprovider || exit 1
run 900 final2_tests.log python -u -m pytest tests -m gpu -q --maxfail=5 --timeout 240 --timeout-method thread -p no:cacheprovider || exit 1
for c in c4 c3; do
  run 200 final2_$c.log python -u bench.py --config $c --no-cpu-baseline --no-other-configs --steps 50 --warmup 5 || exit 1
  MININF_AMD_FINAL_GRADS=0 run 200 final2_${c}_off.log python -u bench.py --config $c --no-cpu-baseline --no-other-configs --steps 50 --warmup 5 || exit 1
done
exit 0
