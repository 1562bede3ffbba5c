#!/bin/bash
# Round 4, eager 4: cached operand keys, early-out side join, plain-tuple broadcast, one-reduction
# guide check; host primitives; breakdowns; the ELBO-path tests.
set -u
mkdir -p gpurun_out
run() { local t=$1; shift; local log=$1; shift; timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; return $rc; }
run 200 e4_micro.log python -u tools/host_micro.py || exit 1
DEEP=1 run 200 e4_breakdown_c2.log python -u tools/eager_breakdown.py c2 200 || exit 1
run 200 e4_breakdown_c2_plain.log python -u tools/eager_breakdown.py c2 300 || exit 1
run 200 e4_breakdown_c4.log python -u tools/eager_breakdown.py c4 200 || exit 1
run 600 e4_tests.log python -u -m pytest -m gpu -q -x --timeout 240 --timeout-method thread -p no:cacheprovider tests/test_gpu_kernels.py tests/test_gpu_parity.py tests/test_gpu_examples.py tests/test_gpu_fused_step.py tests/test_gpu_graph.py || exit 1
exit 0
