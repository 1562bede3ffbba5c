#!/bin/bash
# C5 tail kernels: Adam count modes / workgroup counts (tools/adam_probe.py) and the ELBO
# backward's 16-byte quad path (MININF_AMD_ELBO_QUADS) on the C5 bench, after parity tests of both.
set -u
mkdir -p gpurun_out
L=gpurun_out/r03_tails.log
: > $L
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_optim.py >> $L 2>&1 || { echo "optim rc=$?" >> $L; exit 1; }
MININF_AMD_ADAM_COUNT=2 timeout -k 10 300 $T tests/test_gpu_optim.py >> $L 2>&1 || { echo "optim count2 rc=$?" >> $L; exit 1; }
MININF_AMD_ELBO_QUADS=2 timeout -k 10 600 $T tests/test_gpu_examples.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py >> $L 2>&1 || { echo "quads tests rc=$?" >> $L; exit 1; }
for count in 0 1 2; do
  for blocks in 256 512; do
    MININF_AMD_ADAM_COUNT=$count MININF_AMD_ADAM_BLOCKS=$blocks timeout -k 10 120 python -u tools/adam_probe.py >> $L 2>&1 || { echo "rc=$?" >> $L; exit 1; }
  done
done
B="python -u bench.py --config c5 --steps 40 --warmup 8 --no-cpu-baseline --no-other-configs"
for rep in a b; do
  for q in 0 1 2 4; do
    echo "quads=$q $rep" >> $L
    MININF_AMD_ELBO_QUADS=$q timeout -k 10 200 $B > gpurun_out/r03_tails_q$q$rep.log 2>&1 || { echo "bench rc=$?" >> $L; exit 1; }
    tail -1 gpurun_out/r03_tails_q$q$rep.log | cut -c1-200 >> $L
  done
done
exit 0
