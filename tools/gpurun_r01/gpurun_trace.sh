#!/bin/bash
# Kernel trace of one config (graph replay, as benched): usage gpurun_trace.sh <cfg>
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
cfg=${1:-c2}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_$cfg -o run --output-format csv -- python3 bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/trace_$cfg.log 2>&1
echo "trace rc=$?"
