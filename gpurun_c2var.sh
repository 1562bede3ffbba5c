set -u
mkdir -p gpurun_out
timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/bench_c2.log 2>&1 || exit 1
bash gpurun_trace.sh c2
