#!/bin/bash
# Round 4: C5 fused-draw program knobs at the current code (waves per SIMD, particle-loop unroll,
# LDS tile rows, particle blocks), alternating with the default, one box.
set -u
mkdir -p gpurun_out
run() { local t=$1; shift; local log=$1; shift; timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; return $rc; }
B="python -u bench.py --no-cpu-baseline --no-other-configs --config c5 --steps 96 --warmup 8"
for rep in 1 2; do
  run 120 s5_default_$rep.log $B || exit 1
  MININF_AMD_WAVES_PER_EU=5 run 120 s5_w5_$rep.log $B || exit 1
  MININF_AMD_DRAW_UNROLL=2 run 120 s5_u2_$rep.log $B || exit 1
  MININF_AMD_DRAW_TARGET_BLOCKS=1024 run 120 s5_b1024_$rep.log $B || exit 1
  MININF_AMD_DRAW_TARGET_BLOCKS=4096 run 120 s5_b4096_$rep.log $B || exit 1
done
exit 0
