#!/bin/bash
set -u
mkdir -p gpurun_out
run() { local t=$1; shift; local log=$1; shift; timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; return $rc; }
B="python -u bench.py --steps 40 --warmup 8 --no-cpu-baseline --no-other-configs"
run 200 r03_exp3_p0a.log $B || exit 1
MININF_AMD_BCAST_PREFETCH=1 run 200 r03_exp3_p1a.log $B || exit 1
run 200 r03_exp3_p0b.log $B || exit 1
MININF_AMD_BCAST_PREFETCH=1 run 200 r03_exp3_p1b.log $B || exit 1
exit 0
