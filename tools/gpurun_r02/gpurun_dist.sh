#!/bin/bash
# Sharded path on one GPU: the device two-rank test, then bench with 2 gloo ranks sharing the GPU
set -u
mkdir -p gpurun_out
run() { local t=$1; shift; local log=$1; shift; timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; return $rc; }
run 300 tests_dist.log python -u -m pytest tests/test_gpu_distributed.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider || exit 1
run 200 bench_c2_n1.log python -u bench.py --config ${1:-c2} --steps 30 --warmup 3 --no-cpu-baseline || exit 1
run 300 bench_c2_n2gloo.log python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --config ${1:-c2} --dist-backend gloo --steps 30 --warmup 3 || exit 1
