#!/bin/bash
# Adam workgroup targets 512 (tree) / 384 (v17) / 640 (v18): the probe and the C5 step, plus the
# GPU tests of the long-list reduction (8 particles per block)
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fatal() { [ "$1" -eq 124 ] || [ "$1" -eq 137 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_fused_reduce.py tests/test_gpu_fullsize.py tests/test_gpu_final_grads.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t30_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -1 gpurun_out/t30_tests.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do for v in v1 v17 v18; do
  L=""; [ $v != v1 ] && L=$GRAFT_REPO_ROOT/tools/_timing/$v/libmininf_amd.so
  MININF_AMD_LIB=$L timeout -k 10 60 python3 -u tools/adam_probe.py > gpurun_out/t30_adam.json 2>&1; rc=$?
  echo "$rep $v $(tail -n 1 gpurun_out/t30_adam.json)"; fatal $rc && exit $rc
  MININF_AMD_LIB=$L timeout -k 10 120 python3 -u bench.py --config c5 --steps 240 --no-cpu-baseline --no-other-configs > gpurun_out/t30.json 2> gpurun_out/t30.err; rc=$?
  [ $rc -ne 0 ] && { tail -5 gpurun_out/t30.err; exit $rc; }
  python3 -c "import json; d=json.loads(open('gpurun_out/t30.json').read().strip().splitlines()[-1]); print('$rep $v c5', round(d['ms_per_step']*1e3,2))"
done; done
