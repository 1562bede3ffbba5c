#!/bin/bash
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fatal() { [ "$1" -eq 124 ] || [ "$1" -eq 137 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_fused_reduce.py tests/test_gpu_final_grads.py tests/test_gpu_fused_step.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05_t11_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 gpurun_out/r05_t11_tests.log
[ $rc -ne 0 ] && exit $rc
for c in c2 c4 c5; do
  timeout -k 10 120 python3 -u tools/elbo_timing.py run $c > gpurun_out/etime11_$c.log 2>&1; rc=$?
  echo "etime $c rc=$rc"; tail -2 gpurun_out/etime11_$c.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
timeout -k 10 400 python3 -u bench.py --no-cpu-baseline > gpurun_out/r05_t11_bench.json 2> gpurun_out/r05_t11_bench.err; rc=$?
echo "bench rc=$rc"; fatal $rc && exit $rc
python3 - <<'PY'
import json
for line in open('gpurun_out/r05_t11_bench.json'):
    line=line.strip()
    if not line.startswith('{'): continue
    d=json.loads(line)
    print('c2', d.get('ms_per_step'), d.get('roofline',{}).get('kernel_ms'), d.get('roofline',{}).get('frac'))
    for k, o in (d.get('other_configs') or {}).items():
        print(' ', k, o.get('ms_per_step'), (o.get('roofline') or {}).get('kernel_ms'))
PY
