#!/bin/bash
# Round 6: the C2 site kernel's per-workgroup timeline after the register cut (tools/c2_timeline.py).
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
MININF_AMD_LIB=$GRAFT_REPO_ROOT/tools/_variants/c2tl/libmininf_amd.so timeout -k 10 300 python3 -u tools/c2_timeline.py run gpurun_out/ab15_rows.npy > gpurun_out/ab15_c2_timeline.json 2> gpurun_out/ab15_c2_timeline.err; rc=$?
echo "rc=$rc"; python3 -c "
import json; d=json.load(open('gpurun_out/ab15_c2_timeline.json'))
for k,v in d.items():
    if not k.startswith('last') and not k.startswith('per XCD'): print(k, v)
"
exit $rc
