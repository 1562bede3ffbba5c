set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU --kernel-trace -d gpurun_out/linpmc -o run --output-format csv -- python3 tools/linear_bench.py --reps 10 --shape 128,32,32 --shape 65536,32,32 > gpurun_out/linpmc.log 2>&1
echo "pmc rc=$?"
