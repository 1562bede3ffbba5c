#!/bin/bash
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fatal() { [ "$1" -eq 124 ] || [ "$1" -eq 137 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_optim.py tests/test_gpu_fused_step.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05_t10_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 gpurun_out/r05_t10_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 tools/_timing/stream_probe > gpurun_out/stream_probe4.log 2>&1; echo "stream rc=$?"; tail -2 gpurun_out/stream_probe4.log
for rep in 1 2; do
timeout -k 10 60 python3 -u tools/adam_probe.py > gpurun_out/t10_adam.json 2>&1; rc=$?; echo "adam $(tail -n 1 gpurun_out/t10_adam.json)"; fatal $rc && exit $rc
timeout -k 10 120 python3 -u bench.py --config c5 --no-other-configs --no-cpu-baseline --steps 240 > gpurun_out/t10_c5.json 2> gpurun_out/t10_err.log; rc=$?
if [ $rc -ne 0 ]; then tail -5 gpurun_out/t10_err.log; exit $rc; fi
python3 -c "import json; d=json.loads(open('gpurun_out/t10_c5.json').read().strip().splitlines()[-1]); print('c5', round(d['ms_per_step']*1e3,2), round(d['roofline']['kernel_ms']*1e3,2))"
done
for c in c2 c4; do
  timeout -k 10 120 python3 -u tools/elbo_timing.py run $c > gpurun_out/etime10_$c.log 2>&1; rc=$?
  echo "etime $c rc=$rc"; tail -4 gpurun_out/etime10_$c.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
