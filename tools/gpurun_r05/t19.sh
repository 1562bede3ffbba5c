#!/bin/bash
# the driver's bench command (--steps 20 --warmup 5): graph replays of 5 steps (current choice)
# against one replay of all 20, alternating
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for rep in 1 2 3; do for r in 5 20 10; do
  timeout -k 10 120 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-other-configs --graph-repeat $r > gpurun_out/t19.json 2> gpurun_out/t19.err; rc=$?
  [ $rc -ne 0 ] && { tail -5 gpurun_out/t19.err; exit $rc; }
  python3 -c "import json; d=json.loads(open('gpurun_out/t19.json').read().strip().splitlines()[-1]); print('$rep repeat $r', round(d['ms_per_step']*1e3,2))"
done; done
