#!/bin/bash
# Round 6 A/B 5: C2 chunks sized for the slots left by the side-job workgroups (4064 elements:
# 247 x 4 site + 32 side = 1020 workgroups) against one round of site workgroups alone (3936:
# 1020 site + 32 side, tools/_variants/c2rr).
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fatal() { [ "$1" -eq 124 ] || [ "$1" -eq 137 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_samplers.py tests/test_gpu_parity.py > gpurun_out/ab5_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -1 gpurun_out/ab5_tests.log; fatal $rc && exit $rc
run() { local tag=$1; local cfg=$2; shift 2
  env "$@" timeout -k 10 120 python3 -u bench.py --config $cfg --no-other-configs --no-cpu-baseline --steps 240 > gpurun_out/ab5_$tag.json 2> gpurun_out/ab5_$tag.err; local rc=$?
  echo "$tag rc=$rc $(python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab5_$tag.json').read().strip().splitlines()[-1]); print(round(d['ms_per_step']*1e3,2), round(d['roofline']['kernel_ms']*1e3,2), round(d['roofline']['frac'],3))" 2>&1)"
  if fatal $rc; then exit $rc; fi; }
for r in 1 2 3 4; do
  run c2side$r c2
  run c2rr$r c2 MININF_AMD_LIB=$GRAFT_REPO_ROOT/tools/_variants/c2rr/libmininf_amd.so
done
exit 0
