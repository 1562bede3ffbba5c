#!/bin/bash
# C5 site-program A/B (round 5): the accumulator form of the fused-draw loop against the
# eval form, tile rows / occupancy, particle blocks. Two alternating rounds, one box.
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python3 -u bench.py --config c5 --no-other-configs --no-cpu-baseline --steps 96 --warmup 3"
run() { local tag=$1; shift
  env "$@" timeout -k 10 120 $B > gpurun_out/c5ab_$tag.json 2> gpurun_out/c5ab_$tag.err; local rc=$?
  echo "$tag rc=$rc $(python3 -c "import json,sys; d=json.loads(open('gpurun_out/c5ab_$tag.json').read().strip().splitlines()[-1]); print(round(d['ms_per_step'],5), round(d['roofline']['kernel_ms'],5), d['roofline']['launches_timed'])" 2>&1)"
  if [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi; }
for r in 1 2; do
  run old$r MININF_AMD_ACC_FORM=0
  run acc$r MININF_AMD_ACC_FORM=1
  run t8w5_$r MININF_AMD_TILE_ROWS=8 MININF_AMD_WAVES_PER_EU=5
  run t8w5b1k_$r MININF_AMD_TILE_ROWS=8 MININF_AMD_WAVES_PER_EU=5 MININF_AMD_DRAW_TARGET_BLOCKS=1024
  run t8w5b4k_$r MININF_AMD_TILE_ROWS=8 MININF_AMD_WAVES_PER_EU=5 MININF_AMD_DRAW_TARGET_BLOCKS=4096
  run t8_$r MININF_AMD_TILE_ROWS=8
done
exit 0
