#!/bin/bash
# Round-3 GPU cycle: the -m gpu suite, then bench lines. Each GPU step has its own time limit;
# stop at the first failure. Usage: tools/gpurun_r03/cycle.sh [tests|bench|pg|all]
set -u
mkdir -p gpurun_out
run() { local t=$1; shift; local log=$1; shift; timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; return $rc; }
what=${1:-all}
if [ "$what" = all ] || [ "$what" = tests ]; then
  run 900 r03_tests.log python -u -m pytest tests -m gpu -v --maxfail=5 --timeout 240 --timeout-method thread -p no:cacheprovider ${PYTEST_K:+-k "$PYTEST_K"} || exit 1
fi
if [ "$what" = all ] || [ "$what" = pg ]; then
  run 240 r03_pg_c4.log python -u bench.py --config c4 --process-group --steps 40 --warmup 8 --no-cpu-baseline || exit 1
  run 240 r03_pg_c2.log python -u bench.py --config c2 --process-group --steps 40 --warmup 8 --no-cpu-baseline --no-other-configs || exit 1
fi
if [ "$what" = all ] || [ "$what" = bench ]; then
  run 400 r03_bench.log python -u bench.py || exit 1
fi
exit 0
