#!/bin/bash
set -u
mkdir -p gpurun_out
for c in c3 c4 c2; do timeout -k 10 120 python -u tools/accgrad_probe.py $c > gpurun_out/accgrad_$c.log 2>&1; echo "$c rc=$?"; done
timeout -k 10 200 python -u tools/eager_profile.py c4 100 > gpurun_out/eager_prof_c4.log 2>&1; echo "prof rc=$?"
exit 0
