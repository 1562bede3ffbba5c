#!/bin/bash
# C4-shaped linear site kernel: instruction-fetch and wave-cycle counters (separate passes).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
L=gpurun_out/r03_lin3.log
: > $L
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS --kernel-trace -d gpurun_out/r03_lin3_a -o a --output-format csv -- python3 -u tools/linear_bench.py --only C4 --reps 20 >> $L 2>&1 || { echo "a rc=$?" >> $L; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVES SQ_BUSY_CYCLES --kernel-trace -d gpurun_out/r03_lin3_b -o b --output-format csv -- python3 -u tools/linear_bench.py --only C4 --reps 20 >> $L 2>&1 || { echo "b rc=$?" >> $L; exit 1; }
exit 0
