#!/bin/bash
# PMC counters of the linear-site kernel at the C3 shape (one pass per counter group)
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --kernel-include-regex k_linear -d gpurun_out/pmc_lin$i -o run --output-format csv -- python3 tools/linear_bench.py --only ${1:-C3} --reps 5 > gpurun_out/pmc_lin$i.log 2>&1
  echo "pass $i rc=$?"
done
