#!/bin/bash
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fatal() { [ "$1" -eq 124 ] || [ "$1" -eq 137 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_program_draws.py tests/test_gpu_fusions.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05_t4_new.log 2>&1; rc=$?
echo "new tests rc=$rc"; tail -3 gpurun_out/r05_t4_new.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05_t4_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 gpurun_out/r05_t4_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python3 -u bench.py --config c5 --no-other-configs --no-cpu-baseline --steps 96 > gpurun_out/r05_t4_c5.json 2> gpurun_out/r05_t4_c5.err; rc=$?
echo "c5 rc=$rc"; fatal $rc && exit $rc
python3 -c "import json; d=json.loads(open('gpurun_out/r05_t4_c5.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['roofline']['kernel_ms'], d['config']['fusions'])"
for c in c2 c4 c5 c3; do
  timeout -k 10 120 python3 -u tools/elbo_timing.py run $c > gpurun_out/etime_$c.log 2>&1; rc=$?
  echo "etime $c rc=$rc"; tail -3 gpurun_out/etime_$c.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
timeout -k 10 120 python3 -u tools/graph_branch_probe.py > gpurun_out/branch_probe.log 2>&1; echo "branch rc=$?"; tail -1 gpurun_out/branch_probe.log
timeout -k 10 120 tools/_timing/stream_probe > gpurun_out/stream_probe.log 2>&1; echo "stream rc=$?"; cat gpurun_out/stream_probe.log
