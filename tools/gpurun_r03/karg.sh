#!/bin/bash
# Kernel arguments in device memory (HIP_FORCE_DEV_KERNARG=1) vs the default.
set -u
mkdir -p gpurun_out
L=gpurun_out/r03_karg.log
: > $L
for v in 0 1; do
  echo "HIP_FORCE_DEV_KERNARG=$v" >> $L
  HIP_FORCE_DEV_KERNARG=$v timeout -k 10 120 python -u tools/linear_timing.py run >> $L 2>&1 || { echo "rc=$?" >> $L; exit 1; }
  for c in c4 c2; do
    HIP_FORCE_DEV_KERNARG=$v timeout -k 10 200 python -u bench.py --config $c --steps 100 --warmup 10 --no-cpu-baseline --no-other-configs > gpurun_out/r03_karg_$c$v.log 2>&1 || { echo "bench rc=$?" >> $L; exit 1; }
    echo "$c $(tail -1 gpurun_out/r03_karg_$c$v.log | grep -o '"ms_per_step": [0-9.]*')" >> $L
  done
done
exit 0
