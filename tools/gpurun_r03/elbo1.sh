#!/bin/bash
# ELBO forward final-phase prefetch: tests touching the ELBO kernels, then C2/C4/C5 kernel stats.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
L=gpurun_out/r03_elbo1.log
: > $L
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $T tests/test_gpu_parity.py tests/test_gpu_examples.py tests/test_gpu_fused_reduce.py tests/test_gpu_graph.py tests/test_gpu_prior_fold.py >> $L 2>&1 || { echo "tests rc=$?" >> $L; exit 1; }
for c in c2 c4 c5; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/r03_elbo1_$c -o k --output-format csv -- python3 -u bench.py --config $c --steps 30 --warmup 5 --no-cpu-baseline --no-other-configs > gpurun_out/r03_elbo1_$c.log 2>&1 || { echo "prof rc=$?" >> $L; exit 1; }
  echo "$c $(tail -1 gpurun_out/r03_elbo1_$c.log | grep -o '"ms_per_step": [0-9.]*')" >> $L
done
exit 0
