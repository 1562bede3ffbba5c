#!/bin/bash
# C2 site kernel: particles per lane 4 (tree) against 2 (v12) and 8 (v13), alternating
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for rep in 1 2; do for v in v1 v12 v13; do
  L=""; [ $v != v1 ] && L=$GRAFT_REPO_ROOT/tools/_timing/$v/libmininf_amd.so
  MININF_AMD_LIB=$L timeout -k 10 120 python3 -u bench.py --config c2 --steps 240 --no-cpu-baseline --no-other-configs > gpurun_out/t26.json 2> gpurun_out/t26.err; rc=$?
  [ $rc -ne 0 ] && { tail -5 gpurun_out/t26.err; exit $rc; }
  python3 -c "import json; d=json.loads(open('gpurun_out/t26.json').read().strip().splitlines()[-1]); print('$rep $v', round(d['ms_per_step']*1e3,2), round(d['roofline']['kernel_ms']*1e3,2), d['config']['final_loss'])"
done; done
