set -u
mkdir -p gpurun_out
timeout -k 10 120 python tools/elbo_probe.py > gpurun_out/elbo_probe.log 2>&1 || exit 1
