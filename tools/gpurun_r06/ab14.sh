#!/bin/bash
# Round 6 A/B 14: C2 site kernel after the register cut (the particle-constant segment spread over the
# first chunks, d l / d theta recomputed after the loop: 78 VGPR at 4 particles per lane, 94 at 8):
# particles per lane (MININF_AMD_BCAST_P) x workgroup slots of the chunk plan (MININF_AMD_BCAST_SLOTS).
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fatal() { [ "$1" -eq 124 ] || [ "$1" -eq 137 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
T="tests/test_gpu_samplers.py tests/test_gpu_parity.py tests/test_gpu_kernels.py tests/test_gpu_fusions.py tests/test_gpu_prior_fold.py"
for cfg in "base" "MININF_AMD_BCAST_P=8" "MININF_AMD_BCAST_SLOTS=1536"; do
  e=""; [ "$cfg" != base ] && e="$cfg"
  env $e timeout -k 10 300 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread $T > gpurun_out/ab14_tests.log 2>&1; rc=$?
  echo "tests $cfg rc=$rc $(tail -1 gpurun_out/ab14_tests.log)"; fatal $rc && exit $rc
done
run() { local tag=$1; local cfg=$2; shift 2
  env "$@" timeout -k 10 120 python3 -u bench.py --config $cfg --no-other-configs --no-cpu-baseline --steps 240 > gpurun_out/ab14_$tag.json 2> gpurun_out/ab14_$tag.err; local rc=$?
  echo "$tag rc=$rc $(python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab14_$tag.json').read().strip().splitlines()[-1]); print(round(d['ms_per_step']*1e3,2), round(d['roofline']['kernel_ms']*1e3,2), round(d['roofline']['frac'],3))" 2>&1)"
  if fatal $rc; then exit $rc; fi; }
for r in 1 2; do
  run base$r c2
  run p8_$r c2 MININF_AMD_BCAST_P=8
  run p4s1280_$r c2 MININF_AMD_BCAST_SLOTS=1280
  run p4s1536_$r c2 MININF_AMD_BCAST_SLOTS=1536
  run p8s1280_$r c2 MININF_AMD_BCAST_P=8 MININF_AMD_BCAST_SLOTS=1280
  run old$r c2 MININF_AMD_LIB=$GRAFT_REPO_ROOT/tools/_variants/r06tree/libmininf_amd.so
done
exit 0
