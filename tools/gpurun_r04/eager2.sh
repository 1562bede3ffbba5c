#!/bin/bash
# Round 4, eager 2: lean vmap for the particle trace, lean zero_grad, raw stream handles, the
# validated Beta guide's transform launched directly; the whole GPU suite, eager breakdowns.
set -u
mkdir -p gpurun_out
run() { local t=$1; shift; local log=$1; shift; timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; return $rc; }
run 200 e2_breakdown_c2.log python -u tools/eager_breakdown.py c2 200 || exit 1
run 200 e2_breakdown_c4.log python -u tools/eager_breakdown.py c4 200 || exit 1
run 900 e2_tests.log python -u -m pytest -m gpu -q --timeout 240 --timeout-method thread -p no:cacheprovider tests || exit 1
exit 0
