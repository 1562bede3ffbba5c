#!/bin/bash
# VALU issue counters of each config's dominant kernel (eager steps, one pass per config)
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for c in c2 c3 c5; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/valu_$c -o run --output-format csv -- python3 bench.py --config $c --eager --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/valu_$c.log 2>&1
  echo "valu $c rc=$?"
done
