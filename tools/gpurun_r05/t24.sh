#!/bin/bash
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P="python3 bench.py --no-cpu-baseline --no-other-configs --steps 16 --warmup 2 --warm-ms 0 --config c3"
rm -rf gpurun_out/wait_c3 gpurun_out/vtype_c3
timeout -s KILL 150 rocprofv3 --kernel-include-regex k_linear_mfma --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS GRBM_GUI_ACTIVE -d gpurun_out/wait_c3 -o run --output-format csv -- $P > gpurun_out/wait_c3.log 2>&1; echo "wait_c3 rc=$?"
timeout -s KILL 150 rocprofv3 --kernel-include-regex k_linear_mfma --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE -d gpurun_out/vtype_c3 -o run --output-format csv -- $P > gpurun_out/vtype_c3.log 2>&1; echo "vtype_c3 rc=$?"
