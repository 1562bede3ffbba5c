#!/bin/bash
# Round 4: the whole GPU suite and the default bench line after the last host changes (operand
# collapse fast path, roofline kernel timed after the replays); then the C5 program knob sweep.
set -u
mkdir -p gpurun_out
run() { local t=$1; shift; local log=$1; shift; timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; return $rc; }
run 400 f3_tests.log python -u -m pytest -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_dist_graph.py || exit 1
run 400 f3_bench.log python -u bench.py || exit 1
bash tools/gpurun_r04/c5sweep.sh || exit 1
exit 0
