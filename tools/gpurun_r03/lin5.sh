#!/bin/bash
# Linear-site theta draw with its parameters loaded before the X rows: tests, C4 / C3 bench.
set -u
mkdir -p gpurun_out
run() { local t=$1; shift; local log=$1; shift; timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; return $rc; }
run 900 lin5_tests.log python -u -m pytest tests -m gpu -q --maxfail=5 --timeout 240 --timeout-method thread -p no:cacheprovider || exit 1
B="python -u bench.py --no-cpu-baseline --no-other-configs --steps 50 --warmup 5"
run 200 lin5_c4a.log $B --config c4 || exit 1
run 200 lin5_c4b.log $B --config c4 || exit 1
run 200 lin5_c3.log $B --config c3 || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d gpurun_out/stats5_c4 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-other-configs --config c4 --steps 20 --warmup 3 > gpurun_out/stats5_c4.log 2>&1; echo "stats c4 rc=$?"
exit 0
