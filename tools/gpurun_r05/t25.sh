#!/bin/bash
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for rep in 1 2 3; do for st in 20 240; do
  timeout -k 10 120 python3 -u bench.py --steps $st --warmup 5 --no-cpu-baseline --no-other-configs > gpurun_out/t25.json 2> gpurun_out/t25.err; rc=$?
  [ $rc -ne 0 ] && { tail -5 gpurun_out/t25.err; exit $rc; }
  python3 -c "import json; d=json.loads(open('gpurun_out/t25.json').read().strip().splitlines()[-1]); print('$rep steps $st', round(d['ms_per_step']*1e3,2), round(d['roofline']['kernel_ms']*1e3,2))"
done; done
