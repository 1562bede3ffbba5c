#!/bin/bash
set -u
mkdir -p gpurun_out
for op in cholesky_ex cholesky_ex32 solve_triangular; do
  timeout -k 10 120 python -u tools/capture_probe.py $op >> gpurun_out/r03_probe.log 2>&1; echo "$op rc=$?" >> gpurun_out/r03_probe.log
done
exit 0
