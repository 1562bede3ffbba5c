set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d gpurun_out/linfix -o run --output-format csv -- python3 tools/linear_bench.py --shape 128,32,32 --shape 4096,32,32 --shape 65536,32,32 --reps 20 > gpurun_out/linfix.log 2>&1; echo "rc=$?"
