#!/bin/bash
# Round 4, cycle 8: the linear launch reads the batch counter before the draw's parameters; C4
# A/B and phase stamps; then the round's rocprofv3 evidence (tools/gpurun_r04/prof.sh).
set -u
mkdir -p gpurun_out
run() { local t=$1; shift; local log=$1; shift; timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; return $rc; }
T="python -u -m pytest -m gpu -v --timeout 240 --timeout-method thread -p no:cacheprovider"
run 300 c8_lin.log $T -x tests/test_gpu_linear_draw.py tests/test_gpu_minibatch.py "tests/test_gpu_fullsize.py::test_c4_full_size_bench_configuration" || exit 1
B="python -u bench.py --no-cpu-baseline --no-other-configs --steps 48 --warmup 8"
run 100 c8_c4_a.log $B --config c4 || exit 1
run 100 c8_c4_b.log $B --config c4 || exit 1
run 150 c8_lin_c4.log python -u tools/linear_timing.py bench c4 || exit 1
bash tools/gpurun_r04/prof.sh
exit 0
