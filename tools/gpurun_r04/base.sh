#!/bin/bash
# Round-4 baseline on a fresh box: the new sampler / full-size tests, the full -m gpu suite,
# default bench line.
set -u
mkdir -p gpurun_out
run() { local t=$1; shift; local log=$1; shift; timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; return $rc; }
run 400 base_new.log python -u -m pytest tests/test_gpu_samplers.py "tests/test_gpu_fullsize.py::test_c4_full_size_bench_configuration" -m gpu -v --timeout 240 --timeout-method thread -p no:cacheprovider
run 900 base_tests.log python -u -m pytest tests -m gpu -q --maxfail=5 --timeout 240 --timeout-method thread -p no:cacheprovider --deselect tests/test_gpu_samplers.py --deselect "tests/test_gpu_fullsize.py::test_c4_full_size_bench_configuration" || exit 1
run 400 base_bench.log python -u bench.py || exit 1
exit 0
