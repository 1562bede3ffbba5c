#!/bin/bash
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_peer.py tests/test_native_abi.py tests/test_integration_doc.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r05_t15_peer.log 2>&1; rc=$?
echo "peer tests rc=$rc"; tail -15 gpurun_out/r05_t15_peer.log
exit $rc
