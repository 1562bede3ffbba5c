#!/bin/bash
# C4-shaped linear site kernel: kernel-trace split (kernel vs finalize) and launch variants.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
L=gpurun_out/r03_lin2.log
: > $L
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/r03_lin2_prof -o lin -- python3 -u tools/linear_bench.py --only C4 --reps 50 >> $L 2>&1 || { echo "prof rc=$?" >> $L; exit 1; }
for v in 0 1 2 3 4; do
  MININF_AMD_LINEAR_TUNE=$v timeout -k 10 120 python -u tools/linear_bench.py --only C4 --reps 100 >> $L 2>&1 || { echo "rc=$?" >> $L; exit 1; }
done
exit 0
