#!/bin/bash
# Full GPU suite, C5 packed/unpacked A/B, Adam default probe, default bench.
set -u
mkdir -p gpurun_out
run() { local t=$1; shift; local log=$1; shift; timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; return $rc; }
run 900 r03_tests7.log python -u -m pytest tests -m gpu -v --maxfail=5 --timeout 240 --timeout-method thread -p no:cacheprovider || exit 1
B="python -u bench.py --config c5 --steps 40 --warmup 8 --no-cpu-baseline --no-other-configs"
run 200 r03_c5_packed_a.log $B || exit 1
MININF_AMD_PACKED=0 run 200 r03_c5_scalar_a.log $B || exit 1
run 200 r03_c5_packed_b.log $B || exit 1
MININF_AMD_PACKED=0 run 200 r03_c5_scalar_b.log $B || exit 1
run 120 r03_adam_default.log python -u tools/adam_probe.py || exit 1
run 400 r03_bench7.log python -u bench.py || exit 1
exit 0
