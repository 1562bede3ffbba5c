#!/bin/bash
# Round 6 A/B 12: C2 site kernel priorities: the prologue and the side job at the top level, the
# FMA loop from the level below it, one level down per third (c2prio2); only the side job at the top
# level (c2side3); against the tree. Timeline of c2prio2 (tools/c2_timeline.py).
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fatal() { [ "$1" -eq 124 ] || [ "$1" -eq 137 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
MININF_AMD_LIB=$GRAFT_REPO_ROOT/tools/_variants/c2tlprio2/libmininf_amd.so timeout -k 10 300 python3 -u tools/c2_timeline.py gpurun_out/ab12_rows_prio2.npy > gpurun_out/ab12_tl_prio2.json 2> gpurun_out/ab12_tl_prio2.err; rc=$?
echo "timeline rc=$rc"; fatal $rc && exit $rc
MININF_AMD_LIB=$GRAFT_REPO_ROOT/tools/_variants/c2prio2/libmininf_amd.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_samplers.py tests/test_gpu_parity.py tests/test_gpu_kernels.py tests/test_gpu_fusions.py tests/test_gpu_prior_fold.py > gpurun_out/ab12_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -1 gpurun_out/ab12_tests.log; fatal $rc && exit $rc
run() { local tag=$1; local cfg=$2; shift 2
  env "$@" timeout -k 10 120 python3 -u bench.py --config $cfg --no-other-configs --no-cpu-baseline --steps 240 > gpurun_out/ab12_$tag.json 2> gpurun_out/ab12_$tag.err; local rc=$?
  echo "$tag rc=$rc $(python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab12_$tag.json').read().strip().splitlines()[-1]); print(round(d['ms_per_step']*1e3,2), round(d['roofline']['kernel_ms']*1e3,2), round(d['roofline']['frac'],3))" 2>&1)"
  if fatal $rc; then exit $rc; fi; }
for r in 1 2 3; do
  run c2base$r c2
  run c2prio2_$r c2 MININF_AMD_LIB=$GRAFT_REPO_ROOT/tools/_variants/c2prio2/libmininf_amd.so
  run c2side3_$r c2 MININF_AMD_LIB=$GRAFT_REPO_ROOT/tools/_variants/c2side3/libmininf_amd.so
done
python3 -c "
import json; d=json.load(open('gpurun_out/ab12_tl_prio2.json'))
for k,v in d.items():
    if not k.startswith('last'): print(k, v)
"
exit 0
