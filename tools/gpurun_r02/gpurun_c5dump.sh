set -u
mkdir -p gpurun_out/jit2
PYTEST_X= bash gpurun_r02.sh tests || exit 1
MININF_AMD_JIT_VERBOSE=1 MININF_AMD_JIT_DUMP=gpurun_out/jit2 timeout -k 10 200 python bench.py --config c5 --steps 40 --warmup 8 --no-cpu-baseline --no-other-configs > gpurun_out/bench_c5.log 2>&1 || exit 1
echo "c5 $(tail -1 gpurun_out/bench_c5.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernel_ms"])')"
grep -c "failed to compile" gpurun_out/bench_c5.log
