set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-other-configs > gpurun_out/bench_c2.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/fetch_c2 -o run --output-format csv -- python3 bench.py --eager --steps 4 --warmup 1 --no-cpu-baseline --no-other-configs > gpurun_out/fetch_c2.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/write_c2 -o run --output-format csv -- python3 bench.py --eager --steps 4 --warmup 1 --no-cpu-baseline --no-other-configs > gpurun_out/write_c2.log 2>&1 || exit 1
bash gpurun_trace.sh c2
