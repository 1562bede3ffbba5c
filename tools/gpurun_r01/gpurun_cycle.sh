#!/bin/bash
# One build->measure cycle: GPU parity tests, then benches. Stop at the first failure.
set -u
mkdir -p gpurun_out
run() { local t=$1; shift; local log=$1; shift; timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; return $rc; }
run 500 tests_gpu.log python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider || exit 1
run 200 smoke.log python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
run 200 bench_c2.log python -u bench.py --steps 50 --warmup 5 --no-cpu-baseline || exit 1
run 200 bench_c5.log python -u bench.py --config c5 --steps 10 --warmup 3 --no-cpu-baseline || exit 1
run 200 bench_c3.log python -u bench.py --config c3 --steps 10 --warmup 3 --no-cpu-baseline || exit 1
run 200 bench_c4.log python -u bench.py --config c4 --steps 30 --warmup 5 --no-cpu-baseline || exit 1
exit 0
