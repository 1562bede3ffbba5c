#!/bin/bash
# Round-6 final check on a fresh box: the GPU suite, smoke(), then the default bench line.
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fatal() { [ "$1" -eq 124 ] || [ "$1" -eq 137 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06_final_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 gpurun_out/r06_final_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r06_final_smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -1 gpurun_out/r06_final_smoke.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python3 -u bench.py > gpurun_out/r06_final_bench.json 2> gpurun_out/r06_final_bench.err; rc=$?
echo "bench rc=$rc"; fatal $rc && exit $rc
python3 -c "import json; d=json.loads(open('gpurun_out/r06_final_bench.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['roofline']['frac'], {k: v['ms_per_step'] for k, v in d['other_configs'].items()})"
