#!/bin/bash
# Round 6 check: the C2 launch's span stamps now include the side job's workgroups.
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fatal() { [ "$1" -eq 124 ] || [ "$1" -eq 137 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_samplers.py tests/test_gpu_kernels.py tests/test_gpu_timing_events.py > gpurun_out/ab21_tests.log 2>&1; rc=$?
echo "tests rc=$rc $(tail -1 gpurun_out/ab21_tests.log)"; fatal $rc && exit $rc
for r in 1 2 3; do
  timeout -k 10 120 python3 -u bench.py --config c2 --no-other-configs --no-cpu-baseline --steps 240 > gpurun_out/ab21_c2_$r.json 2> gpurun_out/ab21_c2_$r.err; rc=$?
  echo "c2_$r rc=$rc $(python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab21_c2_$r.json').read().strip().splitlines()[-1]); print(round(d['ms_per_step']*1e3,2), round(d['roofline']['kernel_ms']*1e3,2), round(d['roofline']['frac'],3))" 2>&1)"
  fatal $rc && exit $rc
done
rm -rf gpurun_out/ab21_stats
timeout -s KILL 150 rocprofv3 --kernel-trace --stats -d gpurun_out/ab21_stats -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-other-configs --steps 48 --warmup 3 --warm-ms 20 --config c2 > gpurun_out/ab21_stats.log 2>&1; rc=$?
echo "stats rc=$rc"; grep -h '^{' gpurun_out/ab21_stats.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('stamps', round(d['roofline']['kernel_ms']*1e3,2))"
exit 0
