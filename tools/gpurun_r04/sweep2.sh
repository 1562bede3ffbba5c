#!/bin/bash
# Round 4: the ELBO forward's reduction width (MININF_AMD_ELBO_KRED, particles per reducing block)
# for C2 and the lead-block sizing for C5 (MININF_AMD_ELBO_LEAD=32), at steady clocks, one box.
set -u
mkdir -p gpurun_out
run() { local t=$1; shift; local log=$1; shift; timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; return $rc; }
B="python -u bench.py --no-cpu-baseline --no-other-configs --steps 240 --warmup 8"
for rep in 1 2; do
  for k in 32 16 64; do
    MININF_AMD_ELBO_KRED=$k run 150 w2_c2_k${k}_$rep.log $B --config c2 || exit 1
  done
  for l in 16 32; do
    MININF_AMD_ELBO_LEAD=$l run 150 w2_c5_l${l}_$rep.log $B --config c5 --steps 96 || exit 1
  done
done
exit 0
