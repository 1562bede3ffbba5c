#!/bin/bash
# A/B of library variants (tools/variant_build.py) on one box: bench step times and the Adam probe
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fatal() { [ "$1" -eq 124 ] || [ "$1" -eq 137 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
out=gpurun_out/r05_t6_ab.log
: > $out
lib_of() { if [ "$1" = v1 ]; then echo ""; else echo "$GRAFT_REPO_ROOT/tools/_timing/$1/libmininf_amd.so"; fi; }
for v in v0 v1 v2 v3 v4 v5; do
  MININF_AMD_LIB=$(lib_of $v) timeout -k 10 60 python3 -u tools/adam_probe.py > gpurun_out/t6_adam_$v.json 2>&1; rc=$?
  echo "$v adam $(tail -n 1 gpurun_out/t6_adam_$v.json)" | tee -a $out
  fatal $rc && exit $rc
done
for rep in 1 2; do
  for v in v0 v1 v2 v3 v4 v5; do
    for c in c2 c4 c5; do
      MININF_AMD_LIB=$(lib_of $v) timeout -k 10 120 python3 -u bench.py --config $c --no-other-configs --no-cpu-baseline --steps 240 > gpurun_out/t6_${v}_${c}.json 2> gpurun_out/t6_err.log; rc=$?
      if [ $rc -ne 0 ]; then echo "$v $c rc=$rc" | tee -a $out; tail -5 gpurun_out/t6_err.log; exit $rc; fi
      python3 -c "import json,sys; d=json.loads(open('gpurun_out/t6_${v}_${c}.json').read().strip().splitlines()[-1]); print('$rep $v $c', round(d['ms_per_step']*1e3,2), round(d['roofline']['kernel_ms']*1e3,2))" | tee -a $out
    done
  done
done
