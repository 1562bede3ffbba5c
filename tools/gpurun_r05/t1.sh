#!/bin/bash
# Full GPU suite after the ABI-15 pruning, then the default bench line (kernel time from graph
# replays).
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05_t1_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 gpurun_out/r05_t1_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python3 -u bench.py > gpurun_out/r05_t1_bench.json 2> gpurun_out/r05_t1_bench.err; rc=$?
echo "bench rc=$rc"; exit $rc
