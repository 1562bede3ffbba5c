#!/bin/bash
# targeted re-run: the tests that failed, the capture probe, the N>1 captured bench path
set -u
mkdir -p gpurun_out
run() { local t=$1; shift; local log=$1; shift; timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; return $rc; }
bash tools/gpurun_r03/probe.sh
run 600 r03_tests2.log python -u -m pytest tests/test_gpu_dist_graph.py tests/test_gpu_examples.py tests/test_gpu_optim.py tests/test_gpu_distributed.py tests/test_gpu_graph.py -m gpu -v --timeout 280 --timeout-method thread -p no:cacheprovider
run 240 r03_pg_c4.log python -u bench.py --config c4 --process-group --steps 40 --warmup 8 --no-cpu-baseline || exit 1
run 240 r03_pg_c2.log python -u bench.py --config c2 --process-group --steps 40 --warmup 8 --no-cpu-baseline --no-other-configs || exit 1
run 240 r03_c5_data8.log python -u bench.py --config c5 --shard data --shard-world 8 --steps 10 --warmup 3 --no-cpu-baseline || exit 1
run 240 r03_c5_part.log python -u bench.py --config c5 --steps 10 --warmup 3 --no-cpu-baseline || exit 1
exit 0
