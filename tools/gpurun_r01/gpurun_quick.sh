#!/bin/bash
# Quick check: usage gpurun_quick.sh "<pytest targets>" cfg1 cfg2 ...  (stops at the first failure)
set -u
mkdir -p gpurun_out
run() { local t=$1; shift; local log=$1; shift; timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; return $rc; }
tests=$1; shift
run 400 tests_quick.log python -u -m pytest $tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider || exit 1
for cfg in "$@"; do
  run 200 bench_$cfg.log python -u bench.py --config $cfg --steps 20 --warmup 3 --no-cpu-baseline || exit 1
done
exit 0
