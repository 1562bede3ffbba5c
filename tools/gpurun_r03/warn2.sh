#!/bin/bash
# Which bench config raises the AccumulateGrad stream warning (as an error, with its traceback).
set -u
mkdir -p gpurun_out
for c in c2 c3 c4; do
  timeout -k 10 200 python -u -W "error:The AccumulateGrad:UserWarning" bench.py --config $c --no-other-configs --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/warn2_$c.log 2>&1; echo "$c rc=$?"
done
exit 0
