#!/bin/bash
# Round 6 A/B 3: (a) C2 site kernel with chunks evened out to one round of workgroup slots
# (3936-element chunks, 1020 workgroups) against r05's 4096-element chunks (980 workgroups; variant
# library tools/_variants/c2old); (b) C4's linear kernel taking rows computed one batch ahead
# (mi_rows.next) against drawing them at its start (tools/_variants/c4old). Tests first.
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fatal() { [ "$1" -eq 124 ] || [ "$1" -eq 137 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_samplers.py tests/test_gpu_parity.py tests/test_gpu_kernels.py tests/test_gpu_fusions.py tests/test_gpu_prior_fold.py tests/test_gpu_draw_pairs.py tests/test_gpu_fullsize.py tests/test_gpu_minibatch.py tests/test_gpu_linear_draw.py tests/test_gpu_linear.py tests/test_gpu_graph.py > gpurun_out/ab3_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 gpurun_out/ab3_tests.log; fatal $rc && exit $rc
run() { local tag=$1; local cfg=$2; shift 2
  env "$@" timeout -k 10 120 python3 -u bench.py --config $cfg --no-other-configs --no-cpu-baseline --steps 240 > gpurun_out/ab3_$tag.json 2> gpurun_out/ab3_$tag.err; local rc=$?
  echo "$tag rc=$rc $(python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab3_$tag.json').read().strip().splitlines()[-1]); print(round(d['ms_per_step']*1e3,2), round(d['roofline']['kernel_ms']*1e3,2), round(d['roofline']['frac'],3), d['config']['final_loss'])" 2>&1)"
  if fatal $rc; then exit $rc; fi; }
for r in 1 2 3; do
  run c2new$r c2
  run c2old$r c2 MININF_AMD_LIB=$GRAFT_REPO_ROOT/tools/_variants/c2old/libmininf_amd.so
  run c4new$r c4
  run c4old$r c4 MININF_AMD_LIB=$GRAFT_REPO_ROOT/tools/_variants/c4old/libmininf_amd.so
done
exit 0
