#!/bin/bash
# Prior folding into the linear site (mi_linear.prior): tests, then C3 / C4 with and without it.
set -u
mkdir -p gpurun_out
L=gpurun_out/r03_fold2.log
: > $L
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $T tests/test_gpu_prior_fold.py tests/test_gpu_linear.py tests/test_gpu_minibatch.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py >> $L 2>&1 || { echo "tests rc=$?" >> $L; exit 1; }
for c in c4 c3; do
  for rep in a b; do
    for f in 1 0; do
      MININF_AMD_FOLD_PRIOR=$f timeout -k 10 200 python -u bench.py --config $c --steps 100 --warmup 10 --no-cpu-baseline --no-other-configs > gpurun_out/r03_fold2_$c$f$rep.log 2>&1 || { echo "bench rc=$?" >> $L; exit 1; }
      echo "$c fold=$f $rep $(tail -1 gpurun_out/r03_fold2_$c$f$rep.log | grep -o '"ms_per_step": [0-9.]*')" >> $L
    done
  done
done
exit 0
