set -u
mkdir -p gpurun_out
timeout -k 10 120 python tools/linear_bench.py --shape 128,32,32 --shape 65536,32,32 --shape 262144,32,32 > gpurun_out/linear_c4.log 2>&1 || exit 1
timeout -k 10 600 python bench.py > gpurun_out/bench_default.log 2>&1
echo "default rc=$?"
