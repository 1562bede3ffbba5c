#!/bin/bash
# Eager-step host breakdown and cProfile (C2, C4).
set -u
mkdir -p gpurun_out
run() { local t=$1; shift; local log=$1; shift; timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; return $rc; }
run 200 eager_bd_c2.log python -u tools/eager_breakdown.py c2 100 || exit 1
run 200 eager_prof_c2.log python -u tools/eager_profile.py c2 200 || exit 1
run 200 eager_bd_c4.log python -u tools/eager_breakdown.py c4 100 || exit 1
exit 0
