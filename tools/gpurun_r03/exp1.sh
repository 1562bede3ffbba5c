#!/bin/bash
set -u
mkdir -p gpurun_out
run() { local t=$1; shift; local log=$1; shift; timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; return $rc; }
run 300 r03_exp1_tests.log python -u -m pytest tests/test_gpu_minibatch.py tests/test_gpu_optim.py tests/test_gpu_fullsize.py -m gpu -q --timeout 240 --timeout-method thread -p no:cacheprovider || exit 1
run 200 r03_exp1_c4.log python -u bench.py --config c4 --steps 40 --warmup 8 --no-cpu-baseline || exit 1
run 200 r03_exp1_c5_2048.log python -u bench.py --config c5 --steps 10 --warmup 3 --no-cpu-baseline || exit 1
MININF_AMD_DRAW_TARGET_BLOCKS=1024 run 200 r03_exp1_c5_1024.log python -u bench.py --config c5 --steps 10 --warmup 3 --no-cpu-baseline || exit 1
run 200 r03_exp1_c5d_2048.log python -u bench.py --config c5 --shard data --shard-world 8 --steps 10 --warmup 3 --no-cpu-baseline || exit 1
MININF_AMD_DRAW_TARGET_BLOCKS=1024 run 200 r03_exp1_c5d_1024.log python -u bench.py --config c5 --shard data --shard-world 8 --steps 10 --warmup 3 --no-cpu-baseline || exit 1
exit 0
