#!/bin/bash
# C5: very long reduction lists at 8 particles per block (v15), Adam four quads per lane (v16)
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for rep in 1 2; do for v in v1 v15 v16; do for c in c5 c3; do
  [ $c = c3 ] && [ $v = v16 ] && continue
  L=""; [ $v != v1 ] && L=$GRAFT_REPO_ROOT/tools/_timing/$v/libmininf_amd.so
  MININF_AMD_LIB=$L timeout -k 10 120 python3 -u bench.py --config $c --steps 240 --no-cpu-baseline --no-other-configs > gpurun_out/t29.json 2> gpurun_out/t29.err; rc=$?
  [ $rc -ne 0 ] && { tail -5 gpurun_out/t29.err; exit $rc; }
  python3 -c "import json; d=json.loads(open('gpurun_out/t29.json').read().strip().splitlines()[-1]); print('$rep $v $c', round(d['ms_per_step']*1e3,2), round(d['roofline']['kernel_ms']*1e3,2))"
done; done; done
