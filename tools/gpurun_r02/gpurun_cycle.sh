#!/bin/bash
# One measurement cycle: GPU tests, the default bench run (C2 line + C3/C4/C5 + CPU baseline),
# kernel traces of C2/C4/C5 graph-replay steps.
set -u
mkdir -p gpurun_out
PYTEST_X= bash gpurun_r02.sh tests || exit 1
timeout -k 10 600 python bench.py > gpurun_out/bench_default.log 2>&1; echo "default rc=$?"
bash gpurun_trace.sh c2 c4 c5
