#!/bin/bash
# Round-end evidence: full GPU suite, smoke, default bench (CPU leg included), then the rocprofv3
# passes for profiles/ (kernel-trace stats of every config, HBM bytes, issue counters).
set -u
mkdir -p gpurun_out
run() { local t=$1; shift; local log=$1; shift; timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; return $rc; }
run 900 r03_tests13.log python -u -m pytest tests -m gpu -q --maxfail=5 --timeout 240 --timeout-method thread -p no:cacheprovider || exit 1
run 200 r03_smoke13.log python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
run 400 r03_bench13.log python -u bench.py || exit 1
bash tools/gpurun_r03/prof.sh || exit 1
exit 0
