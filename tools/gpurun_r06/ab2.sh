#!/bin/bash
# Round 6 A/B 2: the data-shard C5 test with the paired loop (JIT log on failure), then C5 base vs
# the paired loop (opaque odd-copy mask), and C3 at 4 vs 3 waves/SIMD. Alternating, one box.
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fatal() { [ "$1" -eq 124 ] || [ "$1" -eq 137 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
MININF_AMD_JIT_VERBOSE=1 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_fullsize.py -k "data_shards" > gpurun_out/ab2_shard.log 2>&1; rc=$?
echo "shard test rc=$rc"; tail -2 gpurun_out/ab2_shard.log; fatal $rc && exit $rc
run() { local tag=$1; local cfg=$2; shift 2
  env "$@" timeout -k 10 120 python3 -u bench.py --config $cfg --no-other-configs --no-cpu-baseline --steps 96 --warmup 3 > gpurun_out/ab2_$tag.json 2> gpurun_out/ab2_$tag.err; local rc=$?
  echo "$tag rc=$rc $(python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab2_$tag.json').read().strip().splitlines()[-1]); print(round(d['ms_per_step']*1e3,2), round(d['roofline']['kernel_ms']*1e3,2), d['config']['final_loss'])" 2>&1)"
  if fatal $rc; then exit $rc; fi; }
for r in 1 2 3; do
  run c5base$r c5 MININF_AMD_DRAW_PAIRS=0
  run c5pair$r c5 MININF_AMD_DRAW_PAIRS=1
  run c3w4_$r c3 MININF_AMD_LINEAR_MINW=4
  run c3w3_$r c3 MININF_AMD_LINEAR_MINW=3
done
exit 0
