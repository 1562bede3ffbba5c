#!/bin/bash
# Round 4 diagnostics: where the C2 / C4 ELBO forward (with Adam) and the C4 linear launch spend
# their time (timing builds: tools/elbo_timing.py, tools/linear_timing.py bench).
set -u
mkdir -p gpurun_out
run() { local t=$1; shift; local log=$1; shift; timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; return $rc; }
run 150 diag_elbo_c2.log python -u tools/elbo_timing.py run c2 || exit 1
run 150 diag_elbo_c4.log python -u tools/elbo_timing.py run c4 || exit 1
run 150 diag_lin_c4.log python -u tools/linear_timing.py bench c4 || exit 1
exit 0
