set -u
mkdir -p gpurun_out
for v in 0 5 0 5; do
  MININF_AMD_BCAST_TUNE=$v timeout -k 10 200 python bench.py --steps 40 --warmup 8 --no-cpu-baseline --no-other-configs > gpurun_out/bench_c2_v$v.log 2>&1 || exit 1
  echo "variant=$v $(tail -1 gpurun_out/bench_c2_v$v.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernel_ms"])')"
done
