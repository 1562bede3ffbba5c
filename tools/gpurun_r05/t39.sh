#!/bin/bash
# The flag mirror's and step counters' argument words read with the shares (tree) vs the previous
# commit (prev): ELBO GPU tests, timing stamps of C2 / C4 / C5, C2 / C4 / C5 bench A/B
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fatal() { [ "$1" -eq 124 ] || [ "$1" -eq 137 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_fused_reduce.py tests/test_gpu_final_grads.py tests/test_gpu_fused_step.py tests/test_gpu_parity.py tests/test_gpu_linear_draw.py tests/test_gpu_fullsize.py tests/test_gpu_program_draws.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t39_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -1 gpurun_out/t39_tests.log; [ $rc -ne 0 ] && exit $rc
for c in c2 c4 c5; do
  timeout -k 10 120 python3 -u tools/elbo_timing.py run $c > gpurun_out/etime39_$c.log 2>&1; rc=$?; echo "etime tree $c rc=$rc"; grep "last block: starts" gpurun_out/etime39_$c.log | tail -1; fatal $rc && exit $rc
done
for rep in 1 2; do for v in tree prev; do
  L=""; [ $v != tree ] && L=$GRAFT_REPO_ROOT/tools/_timing/$v/libmininf_amd.so
  for c in c2 c4 c5; do
    MININF_AMD_LIB=$L timeout -k 10 120 python3 -u bench.py --config $c --steps 480 --no-cpu-baseline --no-other-configs > gpurun_out/t39.json 2> gpurun_out/t39.err; rc=$?
    [ $rc -ne 0 ] && { tail -5 gpurun_out/t39.err; exit $rc; }
    python3 -c "import json; d=json.loads(open('gpurun_out/t39.json').read().strip().splitlines()[-1]); print('$rep $v $c', round(d['ms_per_step']*1e3,2))"
  done
done; done
