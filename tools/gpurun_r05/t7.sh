#!/bin/bash
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_optim.py tests/test_gpu_fused_step.py tests/test_gpu_fused_reduce.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05_t7_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 gpurun_out/r05_t7_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 tools/_timing/stream_probe > gpurun_out/stream_probe2.log 2>&1; echo "stream rc=$?"; cat gpurun_out/stream_probe2.log
