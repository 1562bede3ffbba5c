#!/bin/bash
# C5 fused-draw program: LDS tile rows x occupancy target (and particle unroll); C4 Adam count modes.
set -u
mkdir -p gpurun_out
L=gpurun_out/r03_exp4.log
: > $L
B="python -u bench.py --config c5 --steps 40 --warmup 8 --no-cpu-baseline --no-other-configs"
one() { local tag=$1; shift; env "$@" timeout -k 10 200 $B > gpurun_out/r03_exp4_$tag.log 2>&1 || { echo "$tag rc=$?" >> $L; exit 1; }; echo "$tag $(tail -1 gpurun_out/r03_exp4_$tag.log | cut -c1-330 | grep -o '"ms_per_step": [0-9.]*\|"achieved": [0-9.]*' | tr '\n' ' ')" >> $L; }
for rep in a b; do
  one t16w0$rep MININF_AMD_TILE_ROWS=16
  one t8w0$rep MININF_AMD_TILE_ROWS=8
  one t8w5$rep MININF_AMD_TILE_ROWS=8 MININF_AMD_WAVES_PER_EU=5
  one t8w6$rep MININF_AMD_TILE_ROWS=8 MININF_AMD_WAVES_PER_EU=6
  one t16u2$rep MININF_AMD_TILE_ROWS=16 MININF_AMD_DRAW_UNROLL=2
done
C="python -u bench.py --config c4 --steps 200 --warmup 20 --no-cpu-baseline --no-other-configs"
for rep in a b; do
  for cnt in 1 2; do
    MININF_AMD_ADAM_COUNT=$cnt timeout -k 10 200 $C > gpurun_out/r03_exp4_c4_$cnt$rep.log 2>&1 || { echo "c4 rc=$?" >> $L; exit 1; }
    echo "c4 count=$cnt $rep $(tail -1 gpurun_out/r03_exp4_c4_$cnt$rep.log | grep -o '"ms_per_step": [0-9.]*')" >> $L
  done
done
exit 0
