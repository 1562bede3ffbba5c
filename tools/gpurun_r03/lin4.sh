#!/bin/bash
# Linear-site kernel after the branch-free loads: parity tests, phase timing, C3/C4 bench.
set -u
mkdir -p gpurun_out
L=gpurun_out/r03_lin4.log
: > $L
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $T tests/test_gpu_linear.py tests/test_gpu_minibatch.py tests/test_gpu_fused_reduce.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py >> $L 2>&1 || { echo "tests rc=$?" >> $L; exit 1; }
timeout -k 10 120 python -u tools/linear_timing.py run >> $L 2>&1 || { echo "timing rc=$?" >> $L; exit 1; }
timeout -k 10 120 python -u tools/linear_bench.py --only C4 --reps 100 >> $L 2>&1 || { echo "lb rc=$?" >> $L; exit 1; }
timeout -k 10 120 python -u tools/linear_bench.py --only C3 --reps 30 >> $L 2>&1 || { echo "lb3 rc=$?" >> $L; exit 1; }
for c in c4 c3; do
  timeout -k 10 200 python -u bench.py --config $c --steps 100 --warmup 10 --no-cpu-baseline --no-other-configs > gpurun_out/r03_lin4_$c.log 2>&1 || { echo "bench rc=$?" >> $L; exit 1; }
  echo "$c $(tail -1 gpurun_out/r03_lin4_$c.log | grep -o '"ms_per_step": [0-9.]*')" >> $L
done
exit 0
