#!/bin/bash
# Bench + profile on one MI355X. Each GPU step has its own time limit; stop at the first failure.
set -u
mkdir -p gpurun_out
run() { local t=$1; shift; local log=$1; shift; timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; return $rc; }
run 300 bench_c2.log python bench.py --steps 30 --warmup 5 &&
run 200 bench_c3.log python bench.py --config c3 --steps 10 --warmup 3 --no-cpu-baseline &&
run 200 bench_c5.log python bench.py --config c5 --steps 10 --warmup 3 --no-cpu-baseline &&
run 200 bench_c4.log python bench.py --config c4 --steps 30 --warmup 5 --no-cpu-baseline &&
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
run 300 prof_c2.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2 -o run --output-format csv -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline
