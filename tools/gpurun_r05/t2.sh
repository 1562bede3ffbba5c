#!/bin/bash
# Full GPU suite (ABI 15, accumulator forms), the default bench line, the C5 A/B, then C2's
# issue / wait counters on graph-replayed steps.
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fatal() { [ "$1" -eq 124 ] || [ "$1" -eq 137 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05_t2_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 gpurun_out/r05_t2_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python3 -u bench.py > gpurun_out/r05_t2_bench.json 2> gpurun_out/r05_t2_bench.err; rc=$?
echo "bench rc=$rc"; fatal $rc && exit $rc
bash tools/gpurun_r05/c5ab.sh || exit $?
B="python3 bench.py --no-cpu-baseline --no-other-configs --config c2 --steps 16 --warmup 2 --warm-ms 0"
timeout -s KILL 150 rocprofv3 --kernel-include-regex k_site_bcast --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE -d gpurun_out/r05_wait_c2 -o run --output-format csv -- $B > gpurun_out/r05_wait_c2.log 2>&1; echo "wait_c2 rc=$?"
exit 0
