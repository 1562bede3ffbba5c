#!/bin/bash
# Round 4, cycle 3: why the ELBO-finishing site launches are slow -- A/B of the finishing
# variants against the two-launch paths (C2 group, C4 linear) with kernel-trace stats.
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() { local t=$1; shift; local log=$1; shift; timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; return $rc; }
B="python -u bench.py --no-cpu-baseline --no-other-configs --steps 48 --warmup 8"
run 100 c3_c2_on.log $B --config c2 || exit 1
MININF_AMD_GROUP_ELBO=0 run 100 c3_c2_off.log $B --config c2 || exit 1
run 100 c3_c4_on.log $B --config c4 || exit 1
MININF_AMD_LINEAR_ELBO=0 run 100 c3_c4_off.log $B --config c4 || exit 1
P="python3 bench.py --no-cpu-baseline --no-other-configs --steps 16 --warmup 3"
for c in c2 c4; do
  timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d gpurun_out/c3_stats_${c}_on -o run --output-format csv -- $P --config $c > gpurun_out/c3_stats_${c}_on.log 2>&1 || exit 1
done
MININF_AMD_GROUP_ELBO=0 timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d gpurun_out/c3_stats_c2_off -o run --output-format csv -- $P --config c2 > gpurun_out/c3_stats_c2_off.log 2>&1 || exit 1
MININF_AMD_LINEAR_ELBO=0 timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d gpurun_out/c3_stats_c4_off -o run --output-format csv -- $P --config c4 > gpurun_out/c3_stats_c4_off.log 2>&1 || exit 1
exit 0
