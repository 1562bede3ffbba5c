set -u
mkdir -p gpurun_out
for v in "MININF_AMD_ELBO_KRED=64" "MININF_AMD_ELBO_KRED=32" "MININF_AMD_ELBO_KRED=64" "MININF_AMD_ELBO_KRED=32"; do
  tag=$(echo "$v" | tr ' =' '__')
  env $v timeout -k 10 200 python bench.py --steps 40 --warmup 8 --no-cpu-baseline --no-other-configs > gpurun_out/bench_c2_$tag.log 2>&1 || exit 1
  echo "$v $(tail -1 gpurun_out/bench_c2_$tag.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
done
