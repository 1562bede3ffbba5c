#!/bin/bash
# GPU check: parity tests then smoke; stop on anything worse than a test failure.
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/t1.log 2>&1
rc=$?
echo "pytest exit $rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python __graft_entry__.py --smoke > gpurun_out/smoke.log 2>&1
rc=$?
echo "smoke exit $rc"
exit $rc
