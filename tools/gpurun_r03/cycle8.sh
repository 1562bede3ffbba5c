#!/bin/bash
# Full GPU suite, then C2/C3/C4/C5 graph steps (bench, other configs) and a kernel-stats profile.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local t=$1; shift; local log=$1; shift; timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; return $rc; }
run 900 r03_tests8.log python -u -m pytest tests -m gpu -v --maxfail=5 --timeout 240 --timeout-method thread -p no:cacheprovider || exit 1
run 400 r03_bench8.log python -u bench.py || exit 1
for c in c2 c4 c5; do
  run 300 r03_prof8_$c.log rocprofv3 --kernel-trace --stats -d gpurun_out/r03_prof8_$c -o k --output-format csv -- python3 -u bench.py --config $c --steps 30 --warmup 5 --no-cpu-baseline --no-other-configs || exit 1
done
exit 0
