set -u
mkdir -p gpurun_out
for v in 2048 1024 4096 1024; do
  MININF_AMD_ADAM_CHUNK=$v timeout -k 10 200 python bench.py --config c5 --steps 40 --warmup 8 --no-cpu-baseline --no-other-configs > gpurun_out/bench_c5_adam$v.log 2>&1 || exit 1
  echo "chunk=$v $(tail -1 gpurun_out/bench_c5_adam$v.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
done
