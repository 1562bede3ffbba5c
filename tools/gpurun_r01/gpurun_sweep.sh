#!/bin/bash
# GPU tests, then the default benches, then a row-elements sweep of the C5 site program.
set -u
mkdir -p gpurun_out
run() { local t=$1; shift; local log=$1; shift; timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1; local rc=$?; echo "$log rc=$rc"; return $rc; }
run 400 tests_gpu.log python -m pytest tests -m gpu -x -q || exit 1
run 200 bench_c2.log python bench.py --steps 50 --warmup 5 --no-cpu-baseline || exit 1
run 200 bench_c3.log python bench.py --config c3 --steps 10 --warmup 3 --no-cpu-baseline || exit 1
for e in 4 8 16; do
  MININF_AMD_ROW_ELEMS=$e run 200 sweep_c5_e${e}.log python bench.py --config c5 --steps 10 --warmup 3 --no-cpu-baseline || exit 1
done
run 200 bench_c4.log python bench.py --config c4 --steps 30 --warmup 5 --no-cpu-baseline || exit 1
exit 0
