#!/bin/bash
# Default bench without the CPU leg (eager GC time), then kernel-trace stats of all configs and the
# C4 HBM passes for profiles/.
set -u
mkdir -p gpurun_out
run() { local t=$1; shift; local log=$1; shift; timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; return $rc; }
run 400 r03_bench12.log python -u bench.py --no-cpu-baseline || exit 1
STATS_ONLY=1 bash tools/gpurun_r03/prof.sh || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python3 bench.py --no-cpu-baseline --no-other-configs"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/fetch_c4 -o run --output-format csv -- $B --config c4 --eager --steps 4 --warmup 1 > gpurun_out/fetch_c4.log 2>&1; echo "fetch_c4 rc=$?"
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/write_c4 -o run --output-format csv -- $B --config c4 --eager --steps 4 --warmup 1 > gpurun_out/write_c4.log 2>&1; echo "write_c4 rc=$?"
exit 0
