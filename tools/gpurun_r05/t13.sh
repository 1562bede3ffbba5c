#!/bin/bash
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fatal() { [ "$1" -eq 124 ] || [ "$1" -eq 137 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_fused_reduce.py tests/test_gpu_final_grads.py tests/test_gpu_fused_step.py tests/test_gpu_parity.py tests/test_gpu_linear_draw.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05_t13_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 gpurun_out/r05_t13_tests.log
[ $rc -ne 0 ] && exit $rc
for c in c2 c4 c5; do
  timeout -k 10 120 python3 -u tools/elbo_timing.py run $c > gpurun_out/etime13_$c.log 2>&1; rc=$?
  echo "etime $c rc=$rc"; tail -3 gpurun_out/etime13_$c.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
for c in c2 c4 c5; do
  timeout -k 10 120 python3 -u bench.py --config $c --no-other-configs --no-cpu-baseline --steps 240 > gpurun_out/t13_$c.json 2> gpurun_out/t13_err.log; rc=$?
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/t13_err.log; exit $rc; fi
  python3 -c "import json; d=json.loads(open('gpurun_out/t13_$c.json').read().strip().splitlines()[-1]); print('$c', round(d['ms_per_step']*1e3,2), round(d['roofline']['kernel_ms']*1e3,2))"
done
