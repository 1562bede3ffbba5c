#!/bin/bash
# Round 6: average instruction-fetch latency per kernel (rocprofv3 derived counter InstrFetchLatency
# = accumulate(SQ_IFETCH_LEVEL) / SQ_IFETCH) in the C2, C4 and C5 steps.
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P="python3 bench.py --no-cpu-baseline --no-other-configs --steps 16 --warmup 2 --warm-ms 0"
for c in c2 c4 c5; do
  rm -rf gpurun_out/ifetch_$c
  timeout -s KILL 150 rocprofv3 --pmc InstrFetchLatency SQ_IFETCH SQ_WAVE_CYCLES SQ_WAVES -d gpurun_out/ifetch_$c -o run --output-format csv -- $P --config $c > gpurun_out/ifetch_$c.log 2>&1; rc=$?
  echo "ifetch_$c rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
