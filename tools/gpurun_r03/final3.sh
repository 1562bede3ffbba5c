#!/bin/bash
# A/B of the ELBO forward's final gradients, alternating (box-to-box variance is large).
set -u
mkdir -p gpurun_out
run() { local t=$1; shift; local log=$1; shift; timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; return $rc; }
B="python -u bench.py --no-cpu-baseline --no-other-configs --steps 50 --warmup 5"
for c in c4 c3 c2; do
  run 200 f3_${c}_on1.log $B --config $c || exit 1
  MININF_AMD_FINAL_GRADS=0 run 200 f3_${c}_off.log $B --config $c || exit 1
  run 200 f3_${c}_on2.log $B --config $c || exit 1
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d gpurun_out/stats3_c4 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-other-configs --config c4 --steps 20 --warmup 3 > gpurun_out/stats3_c4.log 2>&1; echo "stats c4 rc=$?"
exit 0
