#!/bin/bash
# Quick check: kernel + parity tests, then one bench config (default c2).
set -u
mkdir -p gpurun_out
run() { local t=$1; shift; local log=$1; shift; timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; return $rc; }
run 400 tests_gpu.log python -m pytest tests -m gpu -x -q || exit 1
run 200 bench_${1:-c2}.log python bench.py --config ${1:-c2} --steps 50 --warmup 5 --no-cpu-baseline || exit 1
exit 0
