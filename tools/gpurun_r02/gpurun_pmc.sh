#!/bin/bash
# SQ / GRBM counters for one bench config (eager steps): usage gpurun_pmc.sh <cfg> <counters...>
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
cfg=$1; shift
timeout -k 10 300 rocprofv3 --pmc "$@" -d gpurun_out/pmc_$cfg -o run --output-format csv -- python3 bench.py --config $cfg --eager --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_$cfg.log 2>&1
echo "pmc rc=$?"
