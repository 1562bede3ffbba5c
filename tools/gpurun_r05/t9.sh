#!/bin/bash
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fatal() { [ "$1" -eq 124 ] || [ "$1" -eq 137 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
for rep in 1 2; do for v in v1 v7 v8 v9; do
  L=""; [ $v != v1 ] && L=$GRAFT_REPO_ROOT/tools/_timing/$v/libmininf_amd.so
  MININF_AMD_LIB=$L timeout -k 10 60 python3 -u tools/adam_probe.py > gpurun_out/t9_adam_$v.json 2>&1; rc=$?
  echo "$rep $v $(tail -n 1 gpurun_out/t9_adam_$v.json)"; fatal $rc && exit $rc
done; done
exit 0
