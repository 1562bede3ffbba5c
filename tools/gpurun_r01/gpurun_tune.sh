#!/bin/bash
# Linear-site kernel variants: usage gpurun_tune.sh <variant ids...>; then the linear parity tests
set -u
mkdir -p gpurun_out
: > gpurun_out/tune.log
for v in "$@"; do
  echo "== variant $v" >> gpurun_out/tune.log
  MININF_AMD_LINEAR_TUNE=$v timeout -k 10 120 python -u tools/linear_bench.py >> gpurun_out/tune.log 2>&1 || exit 1
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_linear.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/tests_linear.log 2>&1; echo "tests rc=$?"
