#!/bin/bash
# Round-6 baseline on a fresh box: the GPU suite, then the default bench line.
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fatal() { [ "$1" -eq 124 ] || [ "$1" -eq 137 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06_base_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 gpurun_out/r06_base_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python3 -u bench.py > gpurun_out/r06_base_bench.json 2> gpurun_out/r06_base_bench.err; rc=$?
echo "bench rc=$rc"; fatal $rc && exit $rc
python3 -c "import json; d=json.loads(open('gpurun_out/r06_base_bench.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['roofline']['frac'], {k: v['ms_per_step'] for k, v in d['other_configs'].items()})"
