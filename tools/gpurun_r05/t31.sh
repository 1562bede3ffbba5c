#!/bin/bash
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 python3 -u tools/elbo_timing.py run c2 > gpurun_out/etime31_c2.log 2>&1; echo "etime rc=$?"; tail -4 gpurun_out/etime31_c2.log
