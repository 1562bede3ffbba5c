#!/bin/bash
# C4 with the linear kernel's launch variants (MININF_AMD_LINEAR_TUNE; 0/1: 512 threads, 256 rows
# per block -> half the partial tiles), and C2 / C4 smoke.
set -u
mkdir -p gpurun_out
L=gpurun_out/r03_tune.log
: > $L
for rep in a b; do
  for v in 3 0 1 2; do
    MININF_AMD_LINEAR_TUNE=$v timeout -k 10 200 python -u bench.py --config c4 --steps 100 --warmup 10 --no-cpu-baseline --no-other-configs > gpurun_out/r03_tune_$v$rep.log 2>&1 || { echo "bench rc=$?" >> $L; exit 1; }
    echo "c4 tune=$v $rep $(tail -1 gpurun_out/r03_tune_$v$rep.log | grep -o '"ms_per_step": [0-9.]*')" >> $L
  done
done
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" >> $L 2>&1 || { echo "smoke rc=$?" >> $L; exit 1; }
exit 0
