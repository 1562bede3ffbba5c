#!/bin/bash
# Round 4, round-end pass: the whole GPU suite, the default bench line, then rocprofv3 kernel-trace
# stats per config and the PMC passes for profiles/ (tools/gpurun_r04/prof.sh).
set -u
mkdir -p gpurun_out
run() { local t=$1; shift; local log=$1; shift; timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; return $rc; }
run 480 f1_tests.log python -u -m pytest -m gpu -q --timeout 240 --timeout-method thread -p no:cacheprovider tests || exit 1
run 400 f1_bench.log python -u bench.py || exit 1
bash tools/gpurun_r04/prof.sh || exit 1
exit 0
