#!/bin/bash
# PMC counters of the C2 BCAST site kernels (scalar-load and LDS variants), eager steps
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
set1="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SMEM SQ_INSTS_LDS GRBM_GUI_ACTIVE GRBM_COUNT"
for v in 1 0; do
  MININF_AMD_BCAST_SMEM=$v timeout -s KILL 120 rocprofv3 --pmc $set1 --kernel-include-regex k_site_bcast -d gpurun_out/pmc_bcast$v -o run --output-format csv -- python3 bench.py --config c2 --eager --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_bcast$v.log 2>&1
  echo "pass $v rc=$?"
done
