#!/bin/bash
# Round 6 A/B 23: k_adam_step with four passes' loads issued together (U = 4: a workgroup's whole
# 4096-element chunk in one memory round trip; tools/_variants/adamu4) against U = 2, in the C5 step.
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fatal() { [ "$1" -eq 124 ] || [ "$1" -eq 137 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
V=$GRAFT_REPO_ROOT/tools/_variants/adamu4/libmininf_amd.so
MININF_AMD_LIB=$V timeout -k 10 300 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_optim.py tests/test_gpu_fused_step.py tests/test_gpu_fullsize.py -k "optim or adam or fused or c5" > gpurun_out/ab23_tests.log 2>&1; rc=$?
echo "tests rc=$rc $(tail -1 gpurun_out/ab23_tests.log)"; fatal $rc && exit $rc
run() { local tag=$1; local cfg=$2; shift 2
  env "$@" timeout -k 10 150 python3 -u bench.py --config $cfg --no-other-configs --no-cpu-baseline --steps 240 > gpurun_out/ab23_$tag.json 2> gpurun_out/ab23_$tag.err; local rc=$?
  echo "$tag rc=$rc $(python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab23_$tag.json').read().strip().splitlines()[-1]); print(round(d['ms_per_step']*1e3,2), round(d['roofline']['kernel_ms']*1e3,2))" 2>&1)"
  if fatal $rc; then exit $rc; fi; }
for r in 1 2 3; do
  run u2_$r c5
  run u4_$r c5 MININF_AMD_LIB=$V
done
for t in u2 u4; do
  rm -rf gpurun_out/ab23_stats_$t; e=""; [ $t = u4 ] && e="MININF_AMD_LIB=$V"
  env $e timeout -s KILL 150 rocprofv3 --kernel-trace --stats -d gpurun_out/ab23_stats_$t -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-other-configs --steps 48 --warmup 3 --warm-ms 20 --config c5 > gpurun_out/ab23_stats_$t.log 2>&1; rc=$?
  echo "stats $t rc=$rc $(grep -h adam_step gpurun_out/ab23_stats_$t/run_kernel_stats.csv | cut -d, -f4-5)"; fatal $rc && exit $rc
done
exit 0
