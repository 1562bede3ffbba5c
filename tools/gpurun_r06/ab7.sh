#!/bin/bash
# Round 6 A/B 7: C2 site kernel with the workgroup's four waves walking the chunk from staggered
# starts (the tree) against walking it in step (tools/_variants/c2norot).
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fatal() { [ "$1" -eq 124 ] || [ "$1" -eq 137 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_samplers.py tests/test_gpu_parity.py tests/test_gpu_kernels.py tests/test_gpu_fusions.py tests/test_gpu_prior_fold.py > gpurun_out/ab7_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -1 gpurun_out/ab7_tests.log; fatal $rc && exit $rc
run() { local tag=$1; local cfg=$2; shift 2
  env "$@" timeout -k 10 120 python3 -u bench.py --config $cfg --no-other-configs --no-cpu-baseline --steps 240 > gpurun_out/ab7_$tag.json 2> gpurun_out/ab7_$tag.err; local rc=$?
  echo "$tag rc=$rc $(python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab7_$tag.json').read().strip().splitlines()[-1]); print(round(d['ms_per_step']*1e3,2), round(d['roofline']['kernel_ms']*1e3,2), round(d['roofline']['frac'],3))" 2>&1)"
  if fatal $rc; then exit $rc; fi; }
for r in 1 2 3 4; do
  run c2stag$r c2
  run c2plain$r c2 MININF_AMD_LIB=$GRAFT_REPO_ROOT/tools/_variants/c2norot/libmininf_amd.so
done
exit 0
