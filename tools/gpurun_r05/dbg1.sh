#!/bin/bash
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
C="--config c4 --steps 4 --warmup 2 --graph-repeat 1 --warm-ms 0 --no-other-configs --no-cpu-baseline"
timeout -k 10 120 python3 -u bench.py --particles-per-gpu 64 $C > gpurun_out/dbg1_one.json 2> gpurun_out/dbg1_one.err; echo "one rc=$?"
tail -30 gpurun_out/dbg1_one.err
timeout -k 10 120 python3 -u bench.py --gpus 2 --dist-backend gloo --particles-per-gpu 32 $C > gpurun_out/dbg1_two.json 2> gpurun_out/dbg1_two.err; echo "two rc=$?"
tail -30 gpurun_out/dbg1_two.err
exit 0
