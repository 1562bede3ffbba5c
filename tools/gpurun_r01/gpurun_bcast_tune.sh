#!/bin/bash
# C2 site kernel: BCAST kernel tests, then the microbenchmark per k_site_bcast_smem variant (MININF_AMD_BCAST_TUNE)
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "bcast or c2 or smoke" > gpurun_out/tests_bcast.log 2>&1; echo "tests rc=$?"; tail -1 gpurun_out/tests_bcast.log
: > gpurun_out/bcast_tune.log
for v in ${@:-0 1 2 3}; do
  echo "== smem variant $v" >> gpurun_out/bcast_tune.log
  MININF_AMD_BCAST_TUNE=$v timeout -k 10 120 python -u tools/bcast_bench.py 2>&1 | grep -v amdgpu.ids >> gpurun_out/bcast_tune.log || exit 1
done
