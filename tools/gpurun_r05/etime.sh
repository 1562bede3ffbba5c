#!/bin/bash
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for c in c2 c4 c5 c3; do
  timeout -k 10 120 python3 -u tools/elbo_timing.py run $c > gpurun_out/etime_$c.log 2>&1; rc=$?
  echo "$c rc=$rc"; tail -3 gpurun_out/etime_$c.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
