#!/bin/bash
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fatal() { [ "$1" -eq 124 ] || [ "$1" -eq 137 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05_final2_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 gpurun_out/r05_final2_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05_final2_smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -1 gpurun_out/r05_final2_smoke.log; fatal $rc && exit $rc
timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r05_final2_bench20.json 2> gpurun_out/r05_final2_bench20.err; rc=$?
echo "bench20 rc=$rc"; fatal $rc && exit $rc
python3 - <<'PY'
import json
d = json.loads([l for l in open('gpurun_out/r05_final2_bench20.json') if l.startswith('{')][-1])
print(round(d['ms_per_step'] * 1e3, 2), d['roofline']['frac'], d['config']['step_mode'],
      {k: round(o['ms_per_step'] * 1e3, 2) for k, o in d['other_configs'].items()})
PY
