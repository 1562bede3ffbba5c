#!/bin/bash
# Round 6 A/B 1: (a) tests of the changed paths -- the paired fused-draw loop on (default), the
# ELBO forward's split finish forced on for the ELBO tests; (b) C5 over (pairs, tile rows, waves per
# EU); (c) C2 / C4 / C5 with the split finish off / on. Alternating rounds on one box.
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fatal() { [ "$1" -eq 124 ] || [ "$1" -eq 137 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
T="python3 -u -m pytest -x -q --timeout 240 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_timing_events.py tests/test_gpu_peer.py tests/test_gpu_fullsize.py tests/test_gpu_program_draws.py tests/test_gpu_final_grads.py tests/test_gpu_fused_step.py tests/test_gpu_parity.py > gpurun_out/ab1_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 gpurun_out/ab1_tests.log; fatal $rc && exit $rc
MININF_AMD_ELBO_SPLIT=1 timeout -k 10 600 $T tests/test_gpu_final_grads.py tests/test_gpu_fused_step.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_fused_reduce.py tests/test_gpu_graph.py tests/test_gpu_optim.py > gpurun_out/ab1_split_tests.log 2>&1; rc=$?
echo "split tests rc=$rc"; tail -2 gpurun_out/ab1_split_tests.log; fatal $rc && exit $rc
run() { local tag=$1; local cfg=$2; shift 2
  env "$@" timeout -k 10 120 python3 -u bench.py --config $cfg --no-other-configs --no-cpu-baseline --steps 96 --warmup 3 > gpurun_out/ab1_$tag.json 2> gpurun_out/ab1_$tag.err; local rc=$?
  echo "$tag rc=$rc $(python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab1_$tag.json').read().strip().splitlines()[-1]); print(round(d['ms_per_step']*1e3,2), round(d['roofline']['kernel_ms']*1e3,2), d['config']['final_loss'])" 2>&1)"
  if fatal $rc; then exit $rc; fi; }
for r in 1 2; do
  run c5base$r c5 MININF_AMD_DRAW_PAIRS=0
  run c5p16$r c5 MININF_AMD_DRAW_PAIRS=1
  run c5p16w4$r c5 MININF_AMD_DRAW_PAIRS=1 MININF_AMD_WAVES_PER_EU=4
  run c5p8w4$r c5 MININF_AMD_DRAW_PAIRS=1 MININF_AMD_TILE_ROWS=8 MININF_AMD_WAVES_PER_EU=4
  run c5s8w5$r c5 MININF_AMD_DRAW_PAIRS=0 MININF_AMD_TILE_ROWS=8 MININF_AMD_WAVES_PER_EU=5
  run c5s8w6$r c5 MININF_AMD_DRAW_PAIRS=0 MININF_AMD_TILE_ROWS=8 MININF_AMD_WAVES_PER_EU=6
done
for r in 1 2; do
  for c in c2 c4 c5; do
    run ${c}split0_$r $c MININF_AMD_ELBO_SPLIT=0
    run ${c}split1_$r $c MININF_AMD_ELBO_SPLIT=1
  done
done
exit 0
