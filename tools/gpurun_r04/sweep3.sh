#!/bin/bash
# Round 4: the long-list reduction width (MININF_AMD_ELBO_KRED_LONG, particles per reducing block
# for ~1000-segment lists) for C4 and C5 at steady clocks, one box.
set -u
mkdir -p gpurun_out
run() { local t=$1; shift; local log=$1; shift; timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; return $rc; }
B="python -u bench.py --no-cpu-baseline --no-other-configs --steps 240 --warmup 8"
for rep in 1 2; do
  for k in 16 8; do
    MININF_AMD_ELBO_KRED_LONG=$k run 150 w3_c4_k${k}_$rep.log $B --config c4 || exit 1
    MININF_AMD_ELBO_KRED_LONG=$k run 150 w3_c5_k${k}_$rep.log $B --config c5 --steps 96 || exit 1
  done
done
exit 0
