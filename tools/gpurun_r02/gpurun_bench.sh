set -u
mkdir -p gpurun_out
timeout -k 10 600 python bench.py > gpurun_out/bench_default.log 2>&1; echo "default rc=$?"
