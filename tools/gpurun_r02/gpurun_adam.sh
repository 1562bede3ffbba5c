#!/bin/bash
# Adam kernel change: its GPU tests, then kernel-trace stats of C5 and C2 graph-replay steps.
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_optim.py tests/test_gpu_graph.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/adam_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
for c in c5 c2; do
  timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d gpurun_out/astats_$c -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-other-configs --config $c --steps 40 --warmup 8 > gpurun_out/astats_$c.log 2>&1; rc=$?; echo "stats $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
