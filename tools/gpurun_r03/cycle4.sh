#!/bin/bash
set -u
mkdir -p gpurun_out
run() { local t=$1; shift; local log=$1; shift; timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; return $rc; }
run 240 r03_gpdebug.log python -u tools/gp_capture_debug.py
run 240 r03_c4.log python -u bench.py --config c4 --steps 40 --warmup 8 --no-cpu-baseline || exit 1
run 240 r03_c4_eager.log python -u tools/eager_breakdown.py c4 50 || exit 1
run 240 r03_c2_eager.log python -u tools/eager_breakdown.py c2 50 || exit 1
exit 0
