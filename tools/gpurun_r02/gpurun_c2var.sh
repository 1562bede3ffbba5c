set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "bcast or c2 or coin or parity or fullsize or graph" > gpurun_out/tests_c2.log 2>&1; echo "tests rc=$?"; tail -1 gpurun_out/tests_c2.log
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 40 --warmup 8 --no-cpu-baseline --no-other-configs > gpurun_out/bench_c2_$i.log 2>&1 || exit 1
  echo "c2 $(tail -1 gpurun_out/bench_c2_$i.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernel_ms"], d["roofline"]["frac"])')"
done
