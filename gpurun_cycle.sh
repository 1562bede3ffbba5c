#!/bin/bash
# One build->measure cycle: GPU parity tests, then benches. Stop at the first failure.
set -u
mkdir -p gpurun_out
run() { local t=$1; shift; local log=$1; shift; timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; return $rc; }
run 400 tests_gpu.log python -m pytest tests -m gpu -x -q || exit 1
run 200 bench_c2.log python bench.py --steps 50 --warmup 5 --no-cpu-baseline || exit 1
run 200 bench_c5.log python bench.py --config c5 --steps 10 --warmup 3 --no-cpu-baseline || exit 1
run 200 bench_c3.log python bench.py --config c3 --steps 10 --warmup 3 --no-cpu-baseline || exit 1
run 200 bench_c4.log python bench.py --config c4 --steps 30 --warmup 5 --no-cpu-baseline || exit 1
exit 0
