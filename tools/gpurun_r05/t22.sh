#!/bin/bash
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for rep in 1 2; do for r in 8 24 12; do for c in c2 c5; do
  timeout -k 10 120 python3 -u bench.py --config $c --steps 240 --no-cpu-baseline --no-other-configs --graph-repeat $r > gpurun_out/t22.json 2> gpurun_out/t22.err; rc=$?
  [ $rc -ne 0 ] && { tail -5 gpurun_out/t22.err; exit $rc; }
  python3 -c "import json; d=json.loads(open('gpurun_out/t22.json').read().strip().splitlines()[-1]); print('$rep repeat $r $c', round(d['ms_per_step']*1e3,2), round(d['roofline']['kernel_ms']*1e3,2))"
done; done; done
