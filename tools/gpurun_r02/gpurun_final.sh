#!/bin/bash
# End-of-round evidence: GPU tests, rocprofv3 stats + PMC passes (profiles/), default bench line.
set -u
mkdir -p gpurun_out
PYTEST_X= bash gpurun_r02.sh tests || exit 1
bash gpurun_prof.sh || exit 1
timeout -k 10 600 python bench.py > gpurun_out/bench_default.log 2>&1; echo "default rc=$?"
