#!/bin/bash
set -u
mkdir -p gpurun_out
run() { local t=$1; shift; local log=$1; shift; timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; return $rc; }
run 150 d3_elbo_c5.log python -u tools/elbo_timing.py run c5 || exit 1
run 150 d3_elbo_c2.log python -u tools/elbo_timing.py run c2 || exit 1
exit 0
