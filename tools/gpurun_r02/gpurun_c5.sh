set -u
mkdir -p gpurun_out
timeout -k 10 200 python bench.py --config c5 --steps 20 --warmup 3 --no-cpu-baseline --no-other-configs > gpurun_out/bench_c5.log 2>&1 || exit 1
bash gpurun_trace.sh c5
