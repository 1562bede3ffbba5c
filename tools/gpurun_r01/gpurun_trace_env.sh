#!/bin/bash
# Kernel trace of one config under extra environment settings: usage gpurun_trace_env.sh <cfg> VAR=value ...
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
cfg=$1; shift
for kv in "$@"; do export "$kv"; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tracex_$cfg -o run --output-format csv -- python3 bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/tracex_$cfg.log 2>&1
echo "trace rc=$?"
