set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "draw or c5 or fullsize or hierarch or parity or graph or example" > gpurun_out/tests_c5.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/tests_c5.log; [ $rc -eq 0 ] || exit 1
for i in 1 2; do
  timeout -k 10 200 python bench.py --config c5 --steps 40 --warmup 8 --no-cpu-baseline --no-other-configs > gpurun_out/bench_c5_$i.log 2>&1 || exit 1
  echo "c5 $(tail -1 gpurun_out/bench_c5_$i.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernel_ms"])')"
done
