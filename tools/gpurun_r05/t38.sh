#!/bin/bash
# The loss and the Beta tails summed through one barrier (tree) vs the previous commit (prev): timing
# stamps and C2 / C4 A/B; then the round's closing checks on the tree: every GPU test, smoke(), the
# default bench line and the kernel-trace stats of C2 / C4 (graph-replayed steps as benched)
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fatal() { [ "$1" -eq 124 ] || [ "$1" -eq 137 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
for c in c2 c4; do
  timeout -k 10 120 python3 -u tools/elbo_timing.py run $c > gpurun_out/etime38_$c.log 2>&1; rc=$?; echo "etime tree $c rc=$rc"; tail -4 gpurun_out/etime38_$c.log; fatal $rc && exit $rc
done
for rep in 1 2; do for v in tree prev; do
  L=""; [ $v != tree ] && L=$GRAFT_REPO_ROOT/tools/_timing/$v/libmininf_amd.so
  for c in c2 c4; do
    MININF_AMD_LIB=$L timeout -k 10 120 python3 -u bench.py --config $c --steps 480 --no-cpu-baseline --no-other-configs > gpurun_out/t38.json 2> gpurun_out/t38.err; rc=$?
    [ $rc -ne 0 ] && { tail -5 gpurun_out/t38.err; exit $rc; }
    python3 -c "import json; d=json.loads(open('gpurun_out/t38.json').read().strip().splitlines()[-1]); print('$rep $v $c', round(d['ms_per_step']*1e3,2))"
  done
done; done
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t38_gpu_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -1 gpurun_out/t38_gpu_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/t38_smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/t38_smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python3 -u bench.py > gpurun_out/r05_final.json 2> gpurun_out/r05_final.err; rc=$?; echo "bench rc=$rc"; tail -c 600 gpurun_out/r05_final.json; fatal $rc && exit $rc
B="python3 bench.py --no-cpu-baseline --no-other-configs"
for c in c2 c4; do
  rm -rf gpurun_out/stats_$c
  timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d gpurun_out/stats_$c -o run --output-format csv -- $B --config $c --steps 20 --warmup 3 > gpurun_out/stats_$c.log 2>&1; rc=$?; echo "stats_$c rc=$rc"; fatal $rc && exit $rc
done
exit 0
