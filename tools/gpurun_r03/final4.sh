#!/bin/bash
# Final gradients without scratch: new tests, full suite, alternating A/B, C4 kernel stats.
set -u
mkdir -p gpurun_out
run() { local t=$1; shift; local log=$1; shift; timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; return $rc; }
run 300 f4_new.log python -u -m pytest tests/test_gpu_final_grads.py tests/test_gpu_linear_draw.py -m gpu -v -x --timeout 120 --timeout-method thread -p no:cacheprovider || exit 1
run 900 f4_tests.log python -u -m pytest tests -m gpu -q --maxfail=5 --timeout 240 --timeout-method thread -p no:cacheprovider || exit 1
B="python -u bench.py --no-cpu-baseline --no-other-configs --steps 50 --warmup 5"
for c in c4 c2 c3; do
  run 200 f4_${c}_on1.log $B --config $c || exit 1
  MININF_AMD_FINAL_GRADS=0 run 200 f4_${c}_off.log $B --config $c || exit 1
  run 200 f4_${c}_on2.log $B --config $c || exit 1
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d gpurun_out/stats4_c4 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-other-configs --config c4 --steps 20 --warmup 3 > gpurun_out/stats4_c4.log 2>&1; echo "stats c4 rc=$?"
exit 0
