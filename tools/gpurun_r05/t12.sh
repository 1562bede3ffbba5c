#!/bin/bash
# A/B: kernel-argument prefetch in the BCAST and linear kernels (v1 = tree) against v10 (without)
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fatal() { [ "$1" -eq 124 ] || [ "$1" -eq 137 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_linear.py tests/test_gpu_linear_draw.py tests/test_gpu_prior_fold.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05_t12_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 gpurun_out/r05_t12_tests.log
[ $rc -ne 0 ] && exit $rc
out=gpurun_out/r05_t12_ab.log; : > $out
for rep in 1 2; do for v in v1 v10; do for c in c2 c4 c3; do
  L=""; [ $v != v1 ] && L=$GRAFT_REPO_ROOT/tools/_timing/$v/libmininf_amd.so
  MININF_AMD_LIB=$L timeout -k 10 120 python3 -u bench.py --config $c --no-other-configs --no-cpu-baseline --steps 240 > gpurun_out/t12_${v}_${c}.json 2> gpurun_out/t12_err.log; rc=$?
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/t12_err.log; exit $rc; fi
  python3 -c "import json; d=json.loads(open('gpurun_out/t12_${v}_${c}.json').read().strip().splitlines()[-1]); print('$rep $v $c', round(d['ms_per_step']*1e3,2), round(d['roofline']['kernel_ms']*1e3,2))" | tee -a $out
done; done; done
