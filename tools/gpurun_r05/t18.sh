#!/bin/bash
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_fused_step.py tests/test_gpu_optim.py tests/test_gpu_final_grads.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05_t18_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 gpurun_out/r05_t18_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python3 -u tools/eager_breakdown.py c2 200 > gpurun_out/r05_eager_c2b.log 2>&1; echo "eager rc=$?"; tail -1 gpurun_out/r05_eager_c2b.log
