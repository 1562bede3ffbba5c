#!/bin/bash
# Round 4, cycle 5: the optimizer step in the ELBO forward (after the lifetime fix), held / held-off
# A/B, timing diagnostics (ELBO forward, C4 linear launch), then the whole -m gpu suite.
set -u
mkdir -p gpurun_out
run() { local t=$1; shift; local log=$1; shift; timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; return $rc; }
T="python -u -m pytest -m gpu -v --timeout 240 --timeout-method thread -p no:cacheprovider"
run 300 c5_step.log $T -x tests/test_gpu_fused_step.py || exit 1
run 300 c5_new.log $T tests/test_gpu_fusions.py tests/test_gpu_samplers.py tests/test_gpu_final_grads.py tests/test_gpu_optim.py tests/test_gpu_linear_elbo.py tests/test_gpu_group_elbo.py
B="python -u bench.py --no-cpu-baseline --no-other-configs --steps 48 --warmup 8"
for c in c2 c4 c5; do
  run 100 c5_ab_${c}_on.log $B --config $c || exit 1
  MININF_AMD_DEFER_STEP=0 run 100 c5_ab_${c}_off.log $B --config $c || exit 1
done
run 150 diag_elbo_c2.log python -u tools/elbo_timing.py run c2 || exit 1
run 150 diag_elbo_c4.log python -u tools/elbo_timing.py run c4 || exit 1
run 150 diag_lin_c4.log python -u tools/linear_timing.py bench c4 || exit 1
run 600 c5_tests.log python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 240 --timeout-method thread -p no:cacheprovider
exit 0
