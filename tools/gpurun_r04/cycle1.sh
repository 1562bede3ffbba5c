#!/bin/bash
# Round 4, cycle 1: the new tests (samplers, full-size C2/C4, fused linear ELBO, ADVICE fixes),
# then the whole -m gpu suite, then the default bench line and a C4 kernel trace.
set -u
mkdir -p gpurun_out
run() { local t=$1; shift; local log=$1; shift; timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; return $rc; }
T="python -u -m pytest -m gpu -v --timeout 240 --timeout-method thread -p no:cacheprovider"
run 400 c1_linelbo.log $T tests/test_gpu_linear_elbo.py tests/test_gpu_group_elbo.py
run 500 c1_new.log $T tests/test_gpu_final_grads.py tests/test_gpu_fusions.py tests/test_gpu_samplers.py tests/test_gpu_fullsize.py tests/test_gpu_minibatch.py tests/test_gpu_graph.py
run 900 c1_tests.log python -u -m pytest tests -m gpu -q --maxfail=8 --timeout 240 --timeout-method thread -p no:cacheprovider || exit 1
run 400 c1_bench.log python -u bench.py || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d gpurun_out/c1_stats_c4 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-other-configs --config c4 --steps 20 --warmup 3 > gpurun_out/c1_stats_c4.log 2>&1; echo "stats c4 rc=$?"
exit 0
