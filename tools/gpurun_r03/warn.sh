#!/bin/bash
# AccumulateGrad stream warning after the warm-up fix: probe, graph tests, default bench.
set -u
mkdir -p gpurun_out
run() { local t=$1; shift; local log=$1; shift; timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; return $rc; }
timeout -k 10 150 python -u tools/accgrad_probe.py c3 > gpurun_out/accgrad5_c3.log 2>&1; echo "probe rc=$?"
run 900 warn_tests.log python -u -m pytest tests -m gpu -q --maxfail=5 --timeout 240 --timeout-method thread -p no:cacheprovider || exit 1
run 400 warn_bench.log python -u bench.py --no-cpu-baseline || exit 1
exit 0
