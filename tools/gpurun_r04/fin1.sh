#!/bin/bash
# Round 4: the optimizer step over a fused-draw factor in the ELBO forward's final-gradient blocks
# (C5); the fused-step tests, then the whole suite, then C5 with and without the fusion.
set -u
mkdir -p gpurun_out
run() { local t=$1; shift; local log=$1; shift; timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; return $rc; }
T="python -u -m pytest -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider"
run 300 g1_fused.log $T -x tests/test_gpu_fused_step.py || exit 1
run 480 g1_tests.log $T tests || exit 1
B="python -u bench.py --no-cpu-baseline --no-other-configs --config c5 --steps 96 --warmup 8"
for rep in 1 2; do
  run 120 g1_c5_on_$rep.log $B || exit 1
  MININF_AMD_ELBO_FIN_ADAM=0 run 120 g1_c5_off_$rep.log $B || exit 1
done
exit 0
