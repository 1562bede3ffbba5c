#!/bin/bash
# Round 4 A/B on one box: the ELBO finished by the site launch (C2 group, C4 linear) and the
# forward's final gradients for C5, against the two-launch paths; eager steps with and without
# the direct gradient accumulation. Graph replay, 50 steps.
set -u
mkdir -p gpurun_out
run() { local t=$1; shift; local log=$1; shift; timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; return $rc; }
B="python -u bench.py --no-cpu-baseline --no-other-configs --steps 50 --warmup 5"
run 150 ab_c2_on1.log $B --config c2 || exit 1
MININF_AMD_GROUP_ELBO=0 run 150 ab_c2_off.log $B --config c2 || exit 1
run 150 ab_c2_on2.log $B --config c2 || exit 1
run 150 ab_c4_on1.log $B --config c4 || exit 1
MININF_AMD_LINEAR_ELBO=0 run 150 ab_c4_off.log $B --config c4 || exit 1
run 150 ab_c4_on2.log $B --config c4 || exit 1
run 150 ab_c5_on1.log $B --config c5 || exit 1
MININF_AMD_FINAL_GRADS=0 run 150 ab_c5_off.log $B --config c5 || exit 1
run 150 ab_c3_on1.log $B --config c3 || exit 1
E="python -u bench.py --no-cpu-baseline --no-other-configs --eager --steps 60 --warmup 10"
run 150 ab_eager_c2_direct.log $E --config c2 || exit 1
MININF_AMD_DIRECT_GRADS=0 run 150 ab_eager_c2_engine.log $E --config c2 || exit 1
run 150 ab_eager_c4_direct.log $E --config c4 || exit 1
run 200 ab_eager_c2_prof.log python -u bench.py --no-cpu-baseline --no-other-configs --eager --steps 20 --warmup 5 --config c2 --profile-host || exit 1
exit 0
