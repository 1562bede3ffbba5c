#!/bin/bash
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fatal() { [ "$1" -eq 124 ] || [ "$1" -eq 137 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
for rep in 1 2; do for v in v1 v11; do
  L=""; [ $v != v1 ] && L=$GRAFT_REPO_ROOT/tools/_timing/$v/libmininf_amd.so
  MININF_AMD_LIB=$L timeout -k 10 60 python3 -u tools/adam_probe.py > gpurun_out/t20_adam_$v.json 2>&1; rc=$?
  echo "$rep $v $(tail -n 1 gpurun_out/t20_adam_$v.json)"; fatal $rc && exit $rc
  MININF_AMD_LIB=$L timeout -k 10 120 python3 -u bench.py --config c5 --no-other-configs --no-cpu-baseline --steps 240 > gpurun_out/t20_${v}.json 2> gpurun_out/t20_err.log; rc=$?
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/t20_err.log; exit $rc; fi
  python3 -c "import json; d=json.loads(open('gpurun_out/t20_${v}.json').read().strip().splitlines()[-1]); print('$rep $v c5', round(d['ms_per_step']*1e3,2), round(d['roofline']['kernel_ms']*1e3,2))"
done; done
