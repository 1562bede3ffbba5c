#!/bin/bash
# Round 4, cycle 2: the one-kernel training step (Adam in the finishing launch, ABI 14) and the
# round's new tests, the default bench line, and the held/held-off A/B of C2 and C4.
set -u
mkdir -p gpurun_out
run() { local t=$1; shift; local log=$1; shift; timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; return $rc; }
T="python -u -m pytest -m gpu -v --timeout 240 --timeout-method thread -p no:cacheprovider"
run 300 c2_step.log $T tests/test_gpu_fused_step.py tests/test_gpu_linear_elbo.py tests/test_gpu_group_elbo.py || exit 1
run 500 c2_new.log $T tests/test_gpu_final_grads.py tests/test_gpu_fusions.py tests/test_gpu_samplers.py tests/test_gpu_fullsize.py tests/test_gpu_minibatch.py tests/test_gpu_graph.py
run 200 c2_bench.log python -u bench.py || exit 1
B="python -u bench.py --no-cpu-baseline --no-other-configs --steps 50 --warmup 5"
run 100 c2_ab_c2_on.log $B --config c2 || exit 1
MININF_AMD_DEFER_STEP=0 run 100 c2_ab_c2_off.log $B --config c2 || exit 1
run 100 c2_ab_c4_on.log $B --config c4 || exit 1
MININF_AMD_DEFER_STEP=0 run 100 c2_ab_c4_off.log $B --config c4 || exit 1
exit 0
