#!/bin/bash
# rocprofv3 evidence for profiles/ (round tag r03): kernel-trace stats of graph-replay steps as
# benched, then separate PMC passes on eager steps: HBM bytes (FETCH_SIZE, WRITE_SIZE), issue
# counters, per-type VALU counters, wave-cycle split. A pass that times out or crashes ends the
# script; an unavailable counter only skips its pass.
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fatal() { [ "$1" -eq 124 ] || [ "$1" -eq 137 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
prof() { local t=$1; shift; local tag=$1; shift
  timeout -s KILL "$t" rocprofv3 "$@" > "gpurun_out/$tag.log" 2>&1; local rc=$?; echo "$tag rc=$rc"
  if fatal $rc; then exit $rc; fi; return $rc; }
B="python3 bench.py --no-cpu-baseline --no-other-configs"
for c in ${CONFIGS:-c2 c3 c4 c5}; do
  prof 240 stats_$c --kernel-trace --stats -d gpurun_out/stats_$c -o run --output-format csv -- $B --config $c --steps 20 --warmup 3 || exit 1
done
[ "${STATS_ONLY:-0}" = 1 ] && exit 0
for c in ${CONFIGS:-c2 c3 c4 c5}; do
  prof 120 fetch_$c --pmc FETCH_SIZE -d gpurun_out/fetch_$c -o run --output-format csv -- $B --config $c --eager --steps 4 --warmup 1
  prof 120 write_$c --pmc WRITE_SIZE -d gpurun_out/write_$c -o run --output-format csv -- $B --config $c --eager --steps 4 --warmup 1
done
for c in c2 c3 c5; do
  prof 120 valu_$c --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/valu_$c -o run --output-format csv -- $B --config $c --eager --steps 3 --warmup 1
  prof 120 vtype_$c --pmc SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 GRBM_GUI_ACTIVE -d gpurun_out/vtype_$c -o run --output-format csv -- $B --config $c --eager --steps 3 --warmup 1
  prof 120 wait_$c --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -d gpurun_out/wait_$c -o run --output-format csv -- $B --config $c --eager --steps 3 --warmup 1
done
exit 0
