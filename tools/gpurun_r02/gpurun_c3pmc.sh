set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE -d gpurun_out/c3pmc -o run --output-format csv -- python3 bench.py --config c3 --eager --steps 3 --warmup 1 --no-cpu-baseline --no-other-configs > gpurun_out/c3pmc.log 2>&1; echo "rc=$?"
