#!/bin/bash
# Round-5 baseline: the default bench line, then C5's site-program issue counters on GRAPH-REPLAYED
# steps (counters from the replayed step, not eager steps).
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fatal() { [ "$1" -eq 124 ] || [ "$1" -eq 137 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
prof() { local t=$1; shift; local tag=$1; shift
  timeout -s KILL "$t" rocprofv3 "$@" > "gpurun_out/$tag.log" 2>&1; local rc=$?; echo "$tag rc=$rc"
  if fatal $rc; then exit $rc; fi; return $rc; }
timeout -k 10 400 python3 -u bench.py > gpurun_out/r05_base.json 2> gpurun_out/r05_base.err; rc=$?
echo "bench rc=$rc"; fatal $rc && exit $rc
B="python3 bench.py --no-cpu-baseline --no-other-configs --config c5 --steps 16 --warmup 2 --warm-ms 0"
prof 150 r05_wait_c5 --kernel-include-regex mi_site_program --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -d gpurun_out/r05_wait_c5 -o run --output-format csv -- $B || exit 1
prof 150 r05_vtype_c5 --kernel-include-regex mi_site_program --pmc SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM GRBM_GUI_ACTIVE -d gpurun_out/r05_vtype_c5 -o run --output-format csv -- $B || exit 1
prof 150 r05_stats_c5 --kernel-trace --stats -d gpurun_out/r05_stats_c5 -o run --output-format csv -- $B || exit 1
exit 0
