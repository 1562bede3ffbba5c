#!/bin/bash
# C5 site program: where the issue slots go. Separate PMC passes on eager
# steps; the JIT sources of the site programs are dumped for offline ISA inspection.
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fatal() { [ "$1" -eq 124 ] || [ "$1" -eq 137 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
prof() { local t=$1; shift; local tag=$1; shift
  timeout -s KILL "$t" rocprofv3 "$@" > "gpurun_out/$tag.log" 2>&1; local rc=$?; echo "$tag rc=$rc"
  if fatal $rc; then exit $rc; fi; return $rc; }
B="python3 bench.py --no-cpu-baseline --no-other-configs --config c5 --eager --steps 3 --warmup 1"
MININF_AMD_JIT_DUMP=gpurun_out/jit_c5 timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-other-configs --config c5 --eager --steps 2 --warmup 1 > gpurun_out/jit_c5.log 2>&1
echo "jit dump rc=$?"
prof 120 r03_wait_c5 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -d gpurun_out/r03_wait_c5 -o run --output-format csv -- $B
prof 120 r03_vtype_c5 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM GRBM_GUI_ACTIVE -d gpurun_out/r03_vtype_c5 -o run --output-format csv -- $B
exit 0
