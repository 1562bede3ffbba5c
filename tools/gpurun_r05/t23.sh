#!/bin/bash
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fatal() { [ "$1" -eq 124 ] || [ "$1" -eq 137 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
for f in a b; do
timeout -k 10 500 python3 -u bench.py > gpurun_out/r05_end_bench_$f.json 2> gpurun_out/r05_end_bench_$f.err; rc=$?
echo "bench rc=$rc"; fatal $rc && exit $rc
python3 - <<PY
import json
d = json.loads([l for l in open('gpurun_out/r05_end_bench_$f.json') if l.startswith('{')][-1])
print(round(d['ms_per_step'] * 1e3, 2), d['roofline']['frac'], d['config']['step_mode'],
      {k: round(o['ms_per_step'] * 1e3, 2) for k, o in d['other_configs'].items()},
      d['config'].get('eager_ms_per_step'), d['cpu_baseline']['value'])
PY
done
