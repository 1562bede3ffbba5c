set -u
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "linear or c3 or c4 or fullsize" > gpurun_out/tests_lin.log 2>&1; echo "tests rc=$?"; tail -1 gpurun_out/tests_lin.log
for v in 3 5 3 5; do
  MININF_AMD_LINEAR_TUNE=$v timeout -k 10 200 python bench.py --config c3 --steps 16 --warmup 4 --no-cpu-baseline --no-other-configs > gpurun_out/bench_c3_v$v.log 2>&1 || exit 1
  echo "variant $v $(tail -1 gpurun_out/bench_c3_v$v.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernel_ms"], d["config"]["final_loss"])')"
done
