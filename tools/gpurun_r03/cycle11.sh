#!/bin/bash
# Full GPU suite, smoke, default bench, eager breakdowns (C2, C4).
set -u
mkdir -p gpurun_out
run() { local t=$1; shift; local log=$1; shift; timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; return $rc; }
run 900 r03_tests11.log python -u -m pytest tests -m gpu -q --maxfail=5 --timeout 240 --timeout-method thread -p no:cacheprovider || exit 1
run 200 r03_smoke11.log python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
run 400 r03_bench11.log python -u bench.py || exit 1
run 200 eager_bd_c2_11.log python -u tools/eager_breakdown.py c2 100 || exit 1
run 200 eager_bd_c4_11.log python -u tools/eager_breakdown.py c4 100 || exit 1
exit 0
