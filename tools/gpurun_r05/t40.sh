#!/bin/bash
# Closing check of the committed tree's library: every GPU test and smoke()
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t40_gpu_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -1 gpurun_out/t40_gpu_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/t40_smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/t40_smoke.log; exit $rc
