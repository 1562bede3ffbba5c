#!/bin/bash
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for c in c2 c3 c5; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$c -o run --output-format csv -- python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof_$c.log 2>&1
  rc=$?; echo "prof $c rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
