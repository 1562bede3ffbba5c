set -u
mkdir -p gpurun_out
for v in 0 2; do
  MININF_AMD_BCAST_TUNE=$v timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-other-configs > gpurun_out/bench_c2_v$v.log 2>&1 || exit 1
done
