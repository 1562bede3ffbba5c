#!/bin/bash
# After releasing the captured step's site tensors: C2 bench with the warning as an error, full
# GPU suite, default bench.
set -u
mkdir -p gpurun_out
run() { local t=$1; shift; local log=$1; shift; timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; return $rc; }
run 200 warn3_c2.log python -u -W "error:The AccumulateGrad:UserWarning" bench.py --config c2 --no-other-configs --no-cpu-baseline --steps 10 --warmup 2
run 900 warn3_tests.log python -u -m pytest tests -m gpu -q --maxfail=5 --timeout 240 --timeout-method thread -p no:cacheprovider || exit 1
run 200 warn3_smoke.log python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
run 400 warn3_bench.log python -u bench.py || exit 1
exit 0
