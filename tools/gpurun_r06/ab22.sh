#!/bin/bash
# Round 6 A/B 22: C5 fused-draw program particle blocks (MININF_AMD_DRAW_GY) 3 (planned) vs 4 / 6 / 8:
# smaller workgroups for the grid's last round against more d loc / d scale partial rows.
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fatal() { [ "$1" -eq 124 ] || [ "$1" -eq 137 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
MININF_AMD_DRAW_GY=6 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_fullsize.py -k c5 tests/test_gpu_program_draws.py > gpurun_out/ab22_tests.log 2>&1; rc=$?
echo "tests rc=$rc $(tail -1 gpurun_out/ab22_tests.log)"; fatal $rc && exit $rc
run() { local tag=$1; local cfg=$2; shift 2
  env "$@" timeout -k 10 150 python3 -u bench.py --config $cfg --no-other-configs --no-cpu-baseline --steps 240 > gpurun_out/ab22_$tag.json 2> gpurun_out/ab22_$tag.err; local rc=$?
  echo "$tag rc=$rc $(python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab22_$tag.json').read().strip().splitlines()[-1]); print(round(d['ms_per_step']*1e3,2), round(d['roofline']['kernel_ms']*1e3,2))" 2>&1)"
  if fatal $rc; then exit $rc; fi; }
for r in 1 2; do
  run gy3_$r c5
  run gy4_$r c5 MININF_AMD_DRAW_GY=4
  run gy6_$r c5 MININF_AMD_DRAW_GY=6
  run gy8_$r c5 MININF_AMD_DRAW_GY=8
done
exit 0
