#!/bin/bash
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 -u tools/eager_profile.py c2 300 > gpurun_out/r05_eager_profile_c2.txt 2>&1; echo "prof rc=$?"; head -60 gpurun_out/r05_eager_profile_c2.txt
