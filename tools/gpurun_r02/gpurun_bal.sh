set -u
mkdir -p gpurun_out
for v in 1 0 1 0; do
  MININF_AMD_ROW_BALANCE=$v timeout -k 10 200 python bench.py --config c5 --steps 20 --warmup 3 --no-cpu-baseline --no-other-configs > gpurun_out/bench_c5_bal$v.log 2>&1 || exit 1
  echo "c5 balance=$v $(tail -1 gpurun_out/bench_c5_bal$v.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernel_ms"], d["roofline"]["frac"])')"
done
