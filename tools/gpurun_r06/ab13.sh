#!/bin/bash
# Round 6 A/B 13: C2 chunk lengths tapered by dispatch rank (MININF_AMD_C2_TAPER, four tiers of
# chunks; sites.hip smem_layout) against uniform chunks; the per-workgroup timeline of the uniform
# plan and of taper A (tools/c2_timeline.py, variant c2tl built from the tree).
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fatal() { [ "$1" -eq 124 ] || [ "$1" -eq 137 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
A=1.25,1.04,0.89,0.82; B=1.15,1.05,0.95,0.85; C=1.35,1.1,0.85,0.7; D=1.1,1.0,1.0,0.9
MININF_AMD_C2_TAPER=$A timeout -k 10 300 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_samplers.py tests/test_gpu_parity.py tests/test_gpu_kernels.py tests/test_gpu_fusions.py tests/test_gpu_prior_fold.py > gpurun_out/ab13_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -1 gpurun_out/ab13_tests.log; fatal $rc && exit $rc
TL="python3 -u tools/c2_timeline.py run"
MININF_AMD_LIB=$GRAFT_REPO_ROOT/tools/_variants/c2tl/libmininf_amd.so timeout -k 10 300 $TL gpurun_out/ab13_rows_u.npy > gpurun_out/ab13_tl_u.json 2> gpurun_out/ab13_tl_u.err; rc=$?
echo "timeline rc=$rc"; fatal $rc && exit $rc
MININF_AMD_C2_TAPER=$A MININF_AMD_LIB=$GRAFT_REPO_ROOT/tools/_variants/c2tl/libmininf_amd.so timeout -k 10 300 $TL gpurun_out/ab13_rows_a.npy > gpurun_out/ab13_tl_a.json 2> gpurun_out/ab13_tl_a.err; rc=$?
echo "timeline rc=$rc"; fatal $rc && exit $rc
run() { local tag=$1; local cfg=$2; shift 2
  env "$@" timeout -k 10 120 python3 -u bench.py --config $cfg --no-other-configs --no-cpu-baseline --steps 240 > gpurun_out/ab13_$tag.json 2> gpurun_out/ab13_$tag.err; local rc=$?
  echo "$tag rc=$rc $(python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab13_$tag.json').read().strip().splitlines()[-1]); print(round(d['ms_per_step']*1e3,2), round(d['roofline']['kernel_ms']*1e3,2), round(d['roofline']['frac'],3))" 2>&1)"
  if fatal $rc; then exit $rc; fi; }
for r in 1 2; do
  run c2u$r c2
  run c2a$r c2 MININF_AMD_C2_TAPER=$A
  run c2b$r c2 MININF_AMD_C2_TAPER=$B
  run c2c$r c2 MININF_AMD_C2_TAPER=$C
  run c2d$r c2 MININF_AMD_C2_TAPER=$D
done
for f in u a; do python3 -c "
import json; d=json.load(open('gpurun_out/ab13_tl_$f.json'))
print('$f', d['kernel_span_us'], d['by dispatch rank (b // 256): n, median prologue, loop, exit; min, max exit'])
"; done
exit 0
