#!/bin/bash
# Round 6: instruction-cache misses per kernel of the C2 and C4 steps (graph replays), one
# rocprofv3 --pmc pass per config.
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P="python3 bench.py --no-cpu-baseline --no-other-configs --steps 16 --warmup 2 --warm-ms 0"
for c in c2 c4 c5; do
  rm -rf gpurun_out/icache_$c
  timeout -s KILL 150 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH GRBM_GUI_ACTIVE -d gpurun_out/icache_$c -o run --output-format csv -- $P --config $c > gpurun_out/icache_$c.log 2>&1; rc=$?
  echo "icache_$c rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
