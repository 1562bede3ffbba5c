#!/bin/bash
# Round 6 A/B 16: C2 after the register cut: the side job at the top priority (MININF_AMD_SIDE_PRIO=1;
# its 32 workgroups now enter at once and were starved until the end) and chunk lengths tapered by
# dispatch rank (MININF_AMD_C2_TAPER) against the tree.
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fatal() { [ "$1" -eq 124 ] || [ "$1" -eq 137 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
T="tests/test_gpu_samplers.py tests/test_gpu_parity.py tests/test_gpu_kernels.py tests/test_gpu_fusions.py tests/test_gpu_prior_fold.py"
for cfg in "MININF_AMD_SIDE_PRIO=1" "MININF_AMD_C2_TAPER=1.4,1.2,0.9,0.5"; do
  env $cfg timeout -k 10 300 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread $T > gpurun_out/ab16_tests.log 2>&1; rc=$?
  echo "tests $cfg rc=$rc $(tail -1 gpurun_out/ab16_tests.log)"; fatal $rc && exit $rc
done
run() { local tag=$1; local cfg=$2; shift 2
  env "$@" timeout -k 10 120 python3 -u bench.py --config $cfg --no-other-configs --no-cpu-baseline --steps 240 > gpurun_out/ab16_$tag.json 2> gpurun_out/ab16_$tag.err; local rc=$?
  echo "$tag rc=$rc $(python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab16_$tag.json').read().strip().splitlines()[-1]); print(round(d['ms_per_step']*1e3,2), round(d['roofline']['kernel_ms']*1e3,2), round(d['roofline']['frac'],3))" 2>&1)"
  if fatal $rc; then exit $rc; fi; }
for r in 1 2; do
  run base$r c2
  run side$r c2 MININF_AMD_SIDE_PRIO=1
  run tE$r c2 MININF_AMD_C2_TAPER=1.3,1.15,0.95,0.6
  run tF$r c2 MININF_AMD_C2_TAPER=1.4,1.2,0.9,0.5
  run tG$r c2 MININF_AMD_C2_TAPER=1.2,1.2,1.0,0.6
  run tEs$r c2 MININF_AMD_C2_TAPER=1.3,1.15,0.95,0.6 MININF_AMD_SIDE_PRIO=1
done
exit 0
