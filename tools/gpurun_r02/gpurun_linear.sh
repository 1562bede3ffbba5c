set -u
mkdir -p gpurun_out
timeout -k 10 120 python tools/linear_bench.py --shape 128,32,32 --shape 65536,32,32 --shape 262144,32,32 > gpurun_out/linear_c4.log 2>&1
