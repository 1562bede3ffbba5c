#!/bin/bash
# C4-shaped linear site kernel: contiguous rows vs gathered rows (sequential / random of 10M).
set -u
mkdir -p gpurun_out
L=gpurun_out/r03_lin.log
: > $L
for g in none seq random; do
  timeout -k 10 120 python -u tools/linear_bench.py --only C4 --gather $g --reps 100 >> $L 2>&1 || { echo "rc=$?" >> $L; exit 1; }
done
exit 0
