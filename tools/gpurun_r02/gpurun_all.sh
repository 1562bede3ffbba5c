set -u
mkdir -p gpurun_out
PYTEST_X= bash gpurun_r02.sh all || exit 1
bash gpurun_trace.sh c4 c5 c3 c2
