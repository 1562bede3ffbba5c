#!/bin/bash
# ELBO forward: 8 vs 16 particles per reducing block for long segment lists (C4, C5).
set -u
mkdir -p gpurun_out
run() { local t=$1; shift; local log=$1; shift; timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; return $rc; }
timeout -k 10 150 python -u tools/accgrad_probe.py c3 > gpurun_out/accgrad4_c3.log 2>&1; echo "probe rc=$?"
B="python -u bench.py --no-cpu-baseline --no-other-configs --steps 50 --warmup 5"
run 300 kred_test.log python -u -m pytest tests/test_gpu_final_grads.py tests/test_gpu_kernels.py -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider || exit 1
MININF_AMD_ELBO_KRED_LONG=8 run 300 kred_test8.log python -u -m pytest tests/test_gpu_final_grads.py tests/test_gpu_kernels.py -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider || exit 1
for c in c4 c5; do
  run 200 kred_${c}_16a.log $B --config $c || exit 1
  MININF_AMD_ELBO_KRED_LONG=8 run 200 kred_${c}_8.log $B --config $c || exit 1
  run 200 kred_${c}_16b.log $B --config $c || exit 1
done
exit 0
