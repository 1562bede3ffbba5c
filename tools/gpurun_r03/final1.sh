#!/bin/bash
# Final guide gradients from the ELBO forward: new tests, full suite, C2 bench A/B.
set -u
mkdir -p gpurun_out
run() { local t=$1; shift; local log=$1; shift; timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; return $rc; }
run 300 final1_new.log python -u -m pytest tests/test_gpu_final_grads.py -m gpu -v -x --timeout 120 --timeout-method thread -p no:cacheprovider || exit 1
run 900 final1_tests.log python -u -m pytest tests -m gpu -q --maxfail=5 --timeout 240 --timeout-method thread -p no:cacheprovider || exit 1
run 200 final1_c2.log python -u bench.py --config c2 --no-cpu-baseline --no-other-configs --steps 50 --warmup 5 || exit 1
MININF_AMD_FINAL_GRADS=0 run 200 final1_c2_off.log python -u bench.py --config c2 --no-cpu-baseline --no-other-configs --steps 50 --warmup 5 || exit 1
run 200 final1_c2b.log python -u bench.py --config c2 --no-cpu-baseline --no-other-configs --steps 50 --warmup 5 || exit 1
exit 0
