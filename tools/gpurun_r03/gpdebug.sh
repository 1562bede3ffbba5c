#!/bin/bash
set -u
mkdir -p gpurun_out
run() { local t=$1; shift; local log=$1; shift; timeout -k 10 "$t" "$@" >> "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; return $rc; }
export GP_DEBUG_BWD=0
GP_DEBUG_TAG=default run 120 r03_gpdebug2.log python -u tools/gp_capture_debug.py || exit 1
GP_DEBUG_TAG=warmup3 GP_DEBUG_WARMUP=3 run 120 r03_gpdebug2.log python -u tools/gp_capture_debug.py || exit 1
GP_DEBUG_TAG=noexp MININF_AMD_DEFER_EXP=0 run 120 r03_gpdebug2.log python -u tools/gp_capture_debug.py || exit 1
GP_DEBUG_TAG=nomvn MININF_AMD_MVN_KERNEL=0 run 120 r03_gpdebug2.log python -u tools/gp_capture_debug.py || exit 1
GP_DEBUG_TAG=nojit MININF_AMD_JIT=0 run 120 r03_gpdebug2.log python -u tools/gp_capture_debug.py || exit 1
exit 0
