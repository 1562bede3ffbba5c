#!/bin/bash
# Round 4, cycle 9: block 0 of the ELBO forward precomputes the tail's trigammas and the Adam bias
# corrections; tests, A/B against cycle 6 numbers, the last block's phases.
set -u
mkdir -p gpurun_out
run() { local t=$1; shift; local log=$1; shift; timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; return $rc; }
T="python -u -m pytest -m gpu -v --timeout 240 --timeout-method thread -p no:cacheprovider"
run 400 c9_tests.log $T -x tests/test_gpu_fused_step.py tests/test_gpu_final_grads.py tests/test_gpu_fusions.py tests/test_gpu_group_elbo.py tests/test_gpu_linear_elbo.py "tests/test_gpu_samplers.py::test_full_size_c2_on_device_draws" "tests/test_gpu_fullsize.py::test_c4_full_size_bench_configuration" tests/test_gpu_kernels.py || exit 1
B="python -u bench.py --no-cpu-baseline --no-other-configs --steps 48 --warmup 8"
for rep in 1 2; do
  for c in c2 c4; do
    run 100 c9_${c}_${rep}.log $B --config $c || exit 1
  done
done
run 150 c9_elbo_c2.log python -u tools/elbo_timing.py run c2 || exit 1
run 150 c9_elbo_c4.log python -u tools/elbo_timing.py run c4 || exit 1
exit 0
