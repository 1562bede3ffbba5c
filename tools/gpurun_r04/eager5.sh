#!/bin/bash
# Round 4, eager 5: bench's eager steps timed without the kernel-event pairs; host primitives;
# callees of the trace's sample and of the ELBO plan's forward.
set -u
mkdir -p gpurun_out
run() { local t=$1; shift; local log=$1; shift; timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; return $rc; }
run 200 e5_micro.log python -u tools/host_micro.py || exit 1
B="python -u bench.py --no-cpu-baseline --no-other-configs"
run 200 e5_bench_1.log $B || exit 1
run 200 e5_bench_2.log $B --steps 150 || exit 1
CALLEES="particles.py.*\(sample\),engine.py.*\(forward\),plan_groups,fold_priors,_fused_beta" run 300 e5_profile_c2.log python -u tools/eager_profile.py c2 300 || exit 1
exit 0
