set -u
mkdir -p gpurun_out
timeout -k 10 200 python bench.py --config c5 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_c5.log 2>&1 || exit 1
MININF_AMD_BCAST_SUFFSTAT=1 timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-other-configs > gpurun_out/bench_c2_suff.log 2>&1 || exit 1
bash gpurun_trace.sh c5
