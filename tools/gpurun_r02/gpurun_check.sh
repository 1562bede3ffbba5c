#!/bin/bash
# GPU tests, then bench lines of the given configs (quick check after a kernel change)
set -u
mkdir -p gpurun_out
PYTEST_X= bash gpurun_r02.sh tests || exit 1
for c in ${CFGS:-c2 c5}; do
  timeout -k 10 200 python bench.py --config $c --steps 40 --warmup 8 --no-cpu-baseline --no-other-configs > gpurun_out/bench_$c.log 2>&1 || exit 1
  echo "$c $(tail -1 gpurun_out/bench_$c.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernel_ms"], d["roofline"]["frac"])')"
done
