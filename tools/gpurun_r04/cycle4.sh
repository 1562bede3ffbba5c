#!/bin/bash
# Round 4, cycle 4: Adam in the ELBO forward's last block (mi_elbo_forward_adam) as the default
# held launch; the finishing site launches opt-in. Tests, then the held / held-off A/B.
set -u
mkdir -p gpurun_out
run() { local t=$1; shift; local log=$1; shift; timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; return $rc; }
T="python -u -m pytest -m gpu -v --timeout 240 --timeout-method thread -p no:cacheprovider"
run 400 c4_step.log $T tests/test_gpu_fused_step.py tests/test_gpu_fusions.py tests/test_gpu_samplers.py tests/test_gpu_final_grads.py tests/test_gpu_optim.py tests/test_gpu_linear_elbo.py tests/test_gpu_group_elbo.py
B="python -u bench.py --no-cpu-baseline --no-other-configs --steps 48 --warmup 8"
for c in c2 c4 c3; do
  run 100 c4_ab_${c}_on.log $B --config $c || exit 1
  MININF_AMD_DEFER_STEP=0 run 100 c4_ab_${c}_off.log $B --config $c || exit 1
done
exit 0
