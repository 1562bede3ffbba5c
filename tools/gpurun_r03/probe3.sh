#!/bin/bash
set -u
mkdir -p gpurun_out
for c in c3 c2; do timeout -k 10 120 python -u tools/accgrad_probe.py $c > gpurun_out/accgrad3_$c.log 2>&1; echo "$c rc=$?"; done
exit 0
