#!/bin/bash
# Round 4, cycle 12: ELBO forward lead-block sizing A/B (MININF_AMD_ELBO_LEAD elements per lane),
# C2 / C4 / C5 step times, interleaved on one box.
set -u
mkdir -p gpurun_out
run() { local t=$1; shift; local log=$1; shift; timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; return $rc; }
B="python -u bench.py --no-cpu-baseline --no-other-configs --steps 48 --warmup 8"
for rep in 1 2; do
  for lead in 4 8 16; do
    for c in c5 c2 c4; do
      MININF_AMD_ELBO_LEAD=$lead run 100 c12_${c}_l${lead}_${rep}.log $B --config $c || exit 1
    done
  done
done
exit 0
