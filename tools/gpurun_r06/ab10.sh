#!/bin/bash
# Round 6: the C2 site kernel's per-workgroup timeline (tools/c2_timeline.py, variant c2tl).
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
MININF_AMD_LIB=$GRAFT_REPO_ROOT/tools/_variants/c2tl/libmininf_amd.so timeout -k 10 300 python3 -u tools/c2_timeline.py gpurun_out/ab10_rows.npy > gpurun_out/ab10_c2_timeline.json 2> gpurun_out/ab10_c2_timeline.err; rc=$?
echo "rc=$rc"; cat gpurun_out/ab10_c2_timeline.json; tail -5 gpurun_out/ab10_c2_timeline.err
exit $rc
