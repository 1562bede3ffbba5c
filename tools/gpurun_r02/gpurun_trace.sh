#!/bin/bash
# Kernel + memory-copy trace of graph-replay steps, per config: usage gpurun_trace.sh c2 [c4 ...]
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for cfg in "$@"; do
  timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/trace_$cfg -o run --output-format csv -- python3 bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline --no-other-configs > gpurun_out/trace_$cfg.log 2>&1
  rc=$?; echo "trace $cfg rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
