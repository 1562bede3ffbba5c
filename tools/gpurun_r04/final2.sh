#!/bin/bash
# Round 4, round-end pass (2): the multi-rank bench tests after the rank-consistent warm-up, the
# default bench line, then rocprofv3 kernel-trace stats per config and the PMC passes.
set -u
mkdir -p gpurun_out
run() { local t=$1; shift; local log=$1; shift; timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; return $rc; }
run 400 f2_tests.log python -u -m pytest -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_dist_graph.py || exit 1
run 400 f2_bench.log python -u bench.py || exit 1
bash tools/gpurun_r04/prof.sh || exit 1
exit 0
