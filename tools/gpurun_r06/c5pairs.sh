#!/bin/bash
# Round 6: the paired fused-draw loop (two particle chains per iteration) -- C5 oracle and fusion
# tests with it on, the timing-event and peer-failure tests, then the C5 A/B over
# (pairs, tile rows, waves per EU), two alternating rounds on one box.
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fatal() { [ "$1" -eq 124 ] || [ "$1" -eq 137 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_timing_events.py tests/test_gpu_peer.py tests/test_gpu_fullsize.py tests/test_gpu_program_draws.py tests/test_gpu_final_grads.py tests/test_gpu_fused_step.py tests/test_gpu_parity.py tests/test_gpu_kernels.py -x -q --timeout 240 --timeout-method thread > gpurun_out/c5p_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 gpurun_out/c5p_tests.log; fatal $rc && exit $rc
B="python3 -u bench.py --config c5 --no-other-configs --no-cpu-baseline --steps 96 --warmup 3"
run() { local tag=$1; shift
  env "$@" timeout -k 10 120 $B > gpurun_out/c5p_$tag.json 2> gpurun_out/c5p_$tag.err; local rc=$?
  echo "$tag rc=$rc $(python3 -c "import json,sys; d=json.loads(open('gpurun_out/c5p_$tag.json').read().strip().splitlines()[-1]); print(round(d['ms_per_step']*1e3,2), round(d['roofline']['kernel_ms']*1e3,2), d['config']['final_loss'])" 2>&1)"
  if fatal $rc; then exit $rc; fi; }
for r in 1 2; do
  run base$r MININF_AMD_DRAW_PAIRS=0
  run p16$r MININF_AMD_DRAW_PAIRS=1
  run p16w4$r MININF_AMD_DRAW_PAIRS=1 MININF_AMD_WAVES_PER_EU=4
  run p8w4$r MININF_AMD_DRAW_PAIRS=1 MININF_AMD_TILE_ROWS=8 MININF_AMD_WAVES_PER_EU=4
  run s8w5$r MININF_AMD_DRAW_PAIRS=0 MININF_AMD_TILE_ROWS=8 MININF_AMD_WAVES_PER_EU=5
  run s8w6$r MININF_AMD_DRAW_PAIRS=0 MININF_AMD_TILE_ROWS=8 MININF_AMD_WAVES_PER_EU=6
  run p8w5$r MININF_AMD_DRAW_PAIRS=1 MININF_AMD_TILE_ROWS=8 MININF_AMD_WAVES_PER_EU=5
done
exit 0
