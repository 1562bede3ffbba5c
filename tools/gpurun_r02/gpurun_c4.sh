set -u
mkdir -p gpurun_out
timeout -k 10 200 python bench.py --config c4 --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/bench_c4.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --config c3 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_c3.log 2>&1 || exit 1
bash gpurun_trace.sh c4
