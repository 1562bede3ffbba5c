#!/bin/bash
# Round-2 GPU cycle: gpu tests, then the bench lines of every config. Each GPU step has its own
# time limit; stop at the first failure.
set -u
mkdir -p gpurun_out
run() { local t=$1; shift; local log=$1; shift; timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; return $rc; }
what=${1:-all}
if [ "$what" = all ] || [ "$what" = tests ]; then
  run 600 tests_gpu.log python -u -m pytest tests -m gpu ${PYTEST_X--x} -v --timeout 120 --timeout-method thread -p no:cacheprovider ${PYTEST_K:+-k "$PYTEST_K"} || exit 1
fi
if [ "$what" = all ] || [ "$what" = bench ]; then
  run 300 bench_c2.log python bench.py --steps 30 --warmup 5 &&
  run 200 bench_c3.log python bench.py --config c3 --steps 10 --warmup 3 --no-cpu-baseline &&
  run 200 bench_c4.log python bench.py --config c4 --steps 30 --warmup 5 --no-cpu-baseline &&
  run 200 bench_c5.log python bench.py --config c5 --steps 10 --warmup 3 --no-cpu-baseline || exit 1
fi
exit 0
