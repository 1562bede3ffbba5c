set -u
mkdir -p gpurun_out
for v in "" "MININF_AMD_DRAW_ELEMS=8" "MININF_AMD_WAVES_PER_EU=5" "MININF_AMD_DRAW_ELEMS=8 MININF_AMD_WAVES_PER_EU=3"; do
  tag=$(echo "$v" | tr ' =' '__')
  env $v timeout -k 10 200 python bench.py --config c5 --steps 20 --warmup 3 --no-cpu-baseline --no-other-configs > gpurun_out/bench_c5_var$tag.log 2>&1 || exit 1
  echo "$v $(tail -1 gpurun_out/bench_c5_var$tag.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["achieved"])')"
done
