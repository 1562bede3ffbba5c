#!/bin/bash
# Adam launch-shape sweep on C5's parameter sizes (tools/adam_probe.py), one process per setting,
# after the bit-identity tests.
set -u
mkdir -p gpurun_out
L=gpurun_out/r03_adam4.log
: > $L
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_optim.py >> $L 2>&1 || { echo "tests rc=$?" >> $L; exit 1; }
MININF_AMD_ADAM_COUNT=2 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_optim.py >> $L 2>&1 || { echo "tests count2 rc=$?" >> $L; exit 1; }
for rep in 1 2; do
  for count in 0 1 2; do
    for blocks in 256 512 1024; do
      MININF_AMD_ADAM_COUNT=$count MININF_AMD_ADAM_BLOCKS=$blocks timeout -k 10 120 python -u tools/adam_probe.py >> $L 2>&1 || { echo "rc=$?" >> $L; exit 1; }
    done
  done
done
exit 0
