#!/bin/bash
# Round 6 A/B 20: C2 site kernel in 512-thread workgroups (MININF_AMD_BCAST_NT=512: 510 workgroups
# of eight waves, two per CU, each chunk's scalar stream shared by eight waves) against 256.
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fatal() { [ "$1" -eq 124 ] || [ "$1" -eq 137 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
T="tests/test_gpu_samplers.py tests/test_gpu_parity.py tests/test_gpu_kernels.py tests/test_gpu_fusions.py tests/test_gpu_prior_fold.py"
MININF_AMD_BCAST_NT=512 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread $T > gpurun_out/ab20_tests.log 2>&1; rc=$?
echo "tests rc=$rc $(tail -1 gpurun_out/ab20_tests.log)"; fatal $rc && exit $rc
run() { local tag=$1; local cfg=$2; shift 2
  env "$@" timeout -k 10 120 python3 -u bench.py --config $cfg --no-other-configs --no-cpu-baseline --steps 240 > gpurun_out/ab20_$tag.json 2> gpurun_out/ab20_$tag.err; local rc=$?
  echo "$tag rc=$rc $(python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab20_$tag.json').read().strip().splitlines()[-1]); print(round(d['ms_per_step']*1e3,2), round(d['roofline']['kernel_ms']*1e3,2), round(d['roofline']['frac'],3))" 2>&1)"
  if fatal $rc; then exit $rc; fi; }
for r in 1 2 3; do
  run nt256_$r c2
  run nt512_$r c2 MININF_AMD_BCAST_NT=512
done
exit 0
