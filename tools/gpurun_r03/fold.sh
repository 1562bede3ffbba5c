#!/bin/bash
# Prior folding (mi_prior): tests, then C2 with and without it.
set -u
mkdir -p gpurun_out
L=gpurun_out/r03_fold.log
: > $L
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $T tests/test_gpu_prior_fold.py tests/test_gpu_parity.py tests/test_gpu_kernels.py tests/test_gpu_examples.py >> $L 2>&1 || { echo "tests rc=$?" >> $L; exit 1; }
B="python -u bench.py --steps 40 --warmup 8 --no-cpu-baseline --no-other-configs"
for rep in a b; do
  for f in 1 0; do
    MININF_AMD_FOLD_PRIOR=$f timeout -k 10 200 $B > gpurun_out/r03_fold_$f$rep.log 2>&1 || { echo "bench rc=$?" >> $L; exit 1; }
    echo "fold=$f $rep $(tail -1 gpurun_out/r03_fold_$f$rep.log | grep -o '"ms_per_step": [0-9.]*')" >> $L
  done
done
exit 0
