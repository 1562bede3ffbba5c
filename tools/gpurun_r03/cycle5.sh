#!/bin/bash
set -u
mkdir -p gpurun_out
run() { local t=$1; shift; local log=$1; shift; timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; return $rc; }
run 900 r03_tests.log python -u -m pytest tests -m gpu -v --maxfail=5 --timeout 240 --timeout-method thread -p no:cacheprovider || exit 1
run 240 r03_c2_eager.log python -u tools/eager_breakdown.py c2 50 || exit 1
run 400 r03_bench.log python -u bench.py || exit 1
exit 0
