#!/bin/bash
# Round 4, cycle 11: fewer, fatter lead blocks in the ELBO forward (C5: 245 instead of 977);
# tests of the ELBO paths, C2 / C4 / C5 step times.
set -u
mkdir -p gpurun_out
run() { local t=$1; shift; local log=$1; shift; timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; return $rc; }
T="python -u -m pytest -m gpu -v --timeout 240 --timeout-method thread -p no:cacheprovider"
run 400 c11_tests.log $T -x tests/test_gpu_final_grads.py tests/test_gpu_fused_step.py tests/test_gpu_fusions.py tests/test_gpu_kernels.py tests/test_gpu_examples.py tests/test_gpu_fused_reduce.py tests/test_gpu_parity.py "tests/test_gpu_fullsize.py::test_c5_fused_draw_full_size_against_oracle" "tests/test_gpu_fullsize.py::test_c5_data_shards_sum_to_the_full_step" || exit 1
B="python -u bench.py --no-cpu-baseline --no-other-configs --steps 48 --warmup 8"
for rep in 1 2; do
  for c in c2 c4 c5; do
    run 100 c11_${c}_${rep}.log $B --config $c || exit 1
  done
done
exit 0
