#!/bin/bash
# Round 6 A/B 25: the linear kernel's stage loads masked at store time (the tree) against masked at
# load time (r06tree), C4 and C3.
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fatal() { [ "$1" -eq 124 ] || [ "$1" -eq 137 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
O=$GRAFT_REPO_ROOT/tools/_variants/r06tree/libmininf_amd.so
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_prior_fold.py tests/test_gpu_linear.py tests/test_gpu_linear_draw.py tests/test_gpu_fullsize.py tests/test_gpu_minibatch.py tests/test_gpu_parity.py > gpurun_out/ab25_tests.log 2>&1; rc=$?
echo "tests rc=$rc $(tail -1 gpurun_out/ab25_tests.log)"; fatal $rc && exit $rc
run() { local tag=$1; local cfg=$2; shift 2
  env "$@" timeout -k 10 150 python3 -u bench.py --config $cfg --no-other-configs --no-cpu-baseline --steps 240 > gpurun_out/ab25_$tag.json 2> gpurun_out/ab25_$tag.err; local rc=$?
  echo "$tag rc=$rc $(python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab25_$tag.json').read().strip().splitlines()[-1]); print(round(d['ms_per_step']*1e3,2), round(d['roofline']['kernel_ms']*1e3,2), round(d['roofline']['frac'],3))" 2>&1)"
  if fatal $rc; then exit $rc; fi; }
for r in 1 2 3 4; do
  run c4new$r c4
  run c4old$r c4 MININF_AMD_LIB=$O
done
for r in 1 2; do
  run c3new$r c3
  run c3old$r c3 MININF_AMD_LIB=$O
done
exit 0
