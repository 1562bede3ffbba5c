#!/bin/bash
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python3 -u tools/eager_breakdown.py c2 200 > gpurun_out/r05_eager_c2.log 2>&1; echo "eager rc=$?"; tail -3 gpurun_out/r05_eager_c2.log
DEEP=1 timeout -k 10 200 python3 -u tools/eager_breakdown.py c2 200 > gpurun_out/r05_eager_c2_deep.log 2>&1; echo "deep rc=$?"; tail -3 gpurun_out/r05_eager_c2_deep.log
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r05_smoke.log 2>&1; echo "smoke rc=$?"; tail -2 gpurun_out/r05_smoke.log
