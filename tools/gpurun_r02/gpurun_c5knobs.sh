#!/bin/bash
# C5 knob sweep: ELBO forward lead-block cap (bench lines only)
set -u
mkdir -p gpurun_out
one() { local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --config ${CFG:-c5} --steps 48 --warmup 8 --no-cpu-baseline --no-other-configs > gpurun_out/k_$tag.log 2>&1 || exit 1
  echo "$tag $(tail -1 gpurun_out/k_$tag.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernel_ms"])')"; }
one base X=1
one l512 MININF_AMD_ELBO_LEAD=512
one l256 MININF_AMD_ELBO_LEAD=256
one l128 MININF_AMD_ELBO_LEAD=128
one base2 X=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for l in 1024 256; do
MININF_AMD_ELBO_LEAD=$l timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d gpurun_out/st5_$l -o run --output-format csv -- python3 bench.py --config c5 --steps 20 --warmup 3 --no-cpu-baseline --no-other-configs > gpurun_out/st5.log 2>&1 || exit 1
done
