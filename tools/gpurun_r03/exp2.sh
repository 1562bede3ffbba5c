#!/bin/bash
set -u
mkdir -p gpurun_out
run() { local t=$1; shift; local log=$1; shift; timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; return $rc; }
run 200 r03_exp2_c4_fused.log python -u bench.py --config c4 --steps 40 --warmup 8 --no-cpu-baseline || exit 1
MININF_AMD_FUSE_ROWS=0 run 200 r03_exp2_c4_plain.log python -u bench.py --config c4 --steps 40 --warmup 8 --no-cpu-baseline || exit 1
run 200 r03_exp2_c4_fused2.log python -u bench.py --config c4 --steps 40 --warmup 8 --no-cpu-baseline || exit 1
exit 0
