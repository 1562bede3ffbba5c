#!/bin/bash
# Round 4, last check after the eager validation-word pool: the whole GPU suite, smoke(), the default
# bench line, kernel-trace stats.
set -u
mkdir -p gpurun_out
run() { local t=$1; shift; local log=$1; shift; timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; return $rc; }
run 480 f7_tests.log python -u -m pytest -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider tests || exit 1
run 200 f7_smoke.log python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
run 400 f7_bench.log python -u bench.py || exit 1
STATS_ONLY=1 bash tools/gpurun_r04/prof.sh || exit 1
exit 0
