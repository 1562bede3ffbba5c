#!/bin/bash
# Round 6 A/B 19: k_adam_step workgroup target (MININF_AMD_ADAM_BLOCKS) in the C5 step: 512 (tree)
# against 768 / 1024 / 384, with the kernel's rocprofv3 trace average per setting.
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fatal() { [ "$1" -eq 124 ] || [ "$1" -eq 137 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
MININF_AMD_ADAM_BLOCKS=1024 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_optim.py tests/test_gpu_fused_step.py > gpurun_out/ab19_tests.log 2>&1; rc=$?
echo "tests rc=$rc $(tail -1 gpurun_out/ab19_tests.log)"; fatal $rc && exit $rc
run() { local tag=$1; local cfg=$2; shift 2
  env "$@" timeout -k 10 150 python3 -u bench.py --config $cfg --no-other-configs --no-cpu-baseline --steps 240 > gpurun_out/ab19_$tag.json 2> gpurun_out/ab19_$tag.err; local rc=$?
  echo "$tag rc=$rc $(python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab19_$tag.json').read().strip().splitlines()[-1]); print(round(d['ms_per_step']*1e3,2), round(d['roofline']['kernel_ms']*1e3,2))" 2>&1)"
  if fatal $rc; then exit $rc; fi; }
for r in 1 2 3; do
  for b in 512 1024 768 384; do run c5b${b}_$r c5 MININF_AMD_ADAM_BLOCKS=$b; done
done
for b in 512 1024; do
  rm -rf gpurun_out/ab19_stats_$b
  MININF_AMD_ADAM_BLOCKS=$b timeout -s KILL 150 rocprofv3 --kernel-trace --stats -d gpurun_out/ab19_stats_$b -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-other-configs --steps 48 --warmup 3 --warm-ms 20 --config c5 > gpurun_out/ab19_stats_$b.log 2>&1; rc=$?
  echo "stats $b rc=$rc $(grep -h adam_step gpurun_out/ab19_stats_$b/run_kernel_stats.csv | cut -d, -f1-4)"; fatal $rc && exit $rc
done
exit 0
