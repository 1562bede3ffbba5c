#!/bin/bash
# Round 6 A/B 9: C2 site kernel variants against the tree: the chunk sum's vector loads issued
# before the per-particle logits (tools/_variants/c2pre); 8 particles per lane at 4 waves per SIMD
# (c2p8: 1010 workgroups of 1984-element chunks, 128 VGPR, 16 B of scratch) and at 3 (c2p8w3: 768
# slots, 2624-element chunks).
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fatal() { [ "$1" -eq 124 ] || [ "$1" -eq 137 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
for v in c2pre c2p8 c2p8w3; do
  MININF_AMD_LIB=$GRAFT_REPO_ROOT/tools/_variants/$v/libmininf_amd.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_samplers.py tests/test_gpu_parity.py tests/test_gpu_kernels.py tests/test_gpu_fusions.py tests/test_gpu_prior_fold.py > gpurun_out/ab9_tests_$v.log 2>&1; rc=$?
  echo "tests $v rc=$rc"; tail -1 gpurun_out/ab9_tests_$v.log; fatal $rc && exit $rc
done
run() { local tag=$1; local cfg=$2; shift 2
  env "$@" timeout -k 10 120 python3 -u bench.py --config $cfg --no-other-configs --no-cpu-baseline --steps 240 > gpurun_out/ab9_$tag.json 2> gpurun_out/ab9_$tag.err; local rc=$?
  echo "$tag rc=$rc $(python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab9_$tag.json').read().strip().splitlines()[-1]); print(round(d['ms_per_step']*1e3,2), round(d['roofline']['kernel_ms']*1e3,2), round(d['roofline']['frac'],3))" 2>&1)"
  if fatal $rc; then exit $rc; fi; }
for r in 1 2 3; do
  run c2base$r c2
  for v in c2pre c2p8 c2p8w3; do
    run $v$r c2 MININF_AMD_LIB=$GRAFT_REPO_ROOT/tools/_variants/$v/libmininf_amd.so
  done
done
exit 0
