#!/bin/bash
# fused-draw site program with the kernel-argument prefetch (v14) against the tree (v1), C5
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
MININF_AMD_LIB=$GRAFT_REPO_ROOT/tools/_timing/v14/libmininf_amd.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_program_draws.py tests/test_gpu_fusions.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t27_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -1 gpurun_out/t27_tests.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2 3; do for v in v1 v14; do
  L=""; [ $v != v1 ] && L=$GRAFT_REPO_ROOT/tools/_timing/$v/libmininf_amd.so
  MININF_AMD_LIB=$L timeout -k 10 120 python3 -u bench.py --config c5 --steps 240 --no-cpu-baseline --no-other-configs > gpurun_out/t27.json 2> gpurun_out/t27.err; rc=$?
  [ $rc -ne 0 ] && { tail -5 gpurun_out/t27.err; exit $rc; }
  python3 -c "import json; d=json.loads(open('gpurun_out/t27.json').read().strip().splitlines()[-1]); print('$rep $v', round(d['ms_per_step']*1e3,2), round(d['roofline']['kernel_ms']*1e3,2))"
done; done
