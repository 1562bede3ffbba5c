#!/bin/bash
# Round 4: the validated eager step keeps its ELBO forward held for Adam; the whole GPU suite,
# eager breakdowns and the default bench line.
set -u
mkdir -p gpurun_out
run() { local t=$1; shift; local log=$1; shift; timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; return $rc; }
run 480 f4_tests.log python -u -m pytest -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider tests || exit 1
run 200 f4_breakdown_c2.log python -u tools/eager_breakdown.py c2 300 || exit 1
run 200 f4_breakdown_c4.log python -u tools/eager_breakdown.py c4 300 || exit 1
run 400 f4_bench.log python -u bench.py || exit 1
exit 0
