#!/bin/bash
# Round 4, eager 3: finer host-time phases of the eager C2 / C4 steps.
set -u
mkdir -p gpurun_out
run() { local t=$1; shift; local log=$1; shift; timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; return $rc; }
DEEP=1 run 200 e3_breakdown_c2.log python -u tools/eager_breakdown.py c2 200 || exit 1
DEEP=1 run 200 e3_breakdown_c4.log python -u tools/eager_breakdown.py c4 200 || exit 1
run 300 e3_profile_c2.log python -u tools/eager_profile.py c2 300 || exit 1
exit 0
