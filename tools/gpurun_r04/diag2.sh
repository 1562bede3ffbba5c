#!/bin/bash
# Round 4 diagnostics 2: the ELBO forward's last-block phases (C2, C4, C5), eager host profile of
# C2 and C4.
set -u
mkdir -p gpurun_out
run() { local t=$1; shift; local log=$1; shift; timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; return $rc; }
run 150 d2_elbo_c2.log python -u tools/elbo_timing.py run c2 || exit 1
run 150 d2_elbo_c4.log python -u tools/elbo_timing.py run c4 || exit 1
run 150 d2_elbo_c5.log python -u tools/elbo_timing.py run c5 || exit 1
run 200 d2_eager_c2.log python -u bench.py --no-cpu-baseline --no-other-configs --eager --steps 20 --warmup 5 --config c2 --profile-host || exit 1
exit 0
