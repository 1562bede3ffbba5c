#!/bin/bash
# Round 4, cycle 6: Adam bias corrections precomputed in parallel lanes of the ELBO forward's last
# block; sampler-test fixes; held / held-off A/B (alternating, twice); reduction-width A/B for the
# ELBO forward (MININF_AMD_ELBO_KRED for C2, _KRED_LONG for C4).
set -u
mkdir -p gpurun_out
run() { local t=$1; shift; local log=$1; shift; timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; return $rc; }
T="python -u -m pytest -m gpu -v --timeout 240 --timeout-method thread -p no:cacheprovider"
run 300 c6_step.log $T -x tests/test_gpu_fused_step.py tests/test_gpu_samplers.py tests/test_gpu_final_grads.py || exit 1
B="python -u bench.py --no-cpu-baseline --no-other-configs --steps 48 --warmup 8"
for rep in 1 2; do
  for c in c2 c4; do
    run 100 c6_ab_${c}_on${rep}.log $B --config $c || exit 1
    MININF_AMD_DEFER_STEP=0 run 100 c6_ab_${c}_off${rep}.log $B --config $c || exit 1
  done
done
MININF_AMD_ELBO_KRED_LONG=8 run 100 c6_kl8_c4.log $B --config c4 || exit 1
MININF_AMD_ELBO_KRED=16 run 100 c6_kr16_c2.log $B --config c2 || exit 1
MININF_AMD_ELBO_KRED=64 run 100 c6_kr64_c2.log $B --config c2 || exit 1
exit 0
