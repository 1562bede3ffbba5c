#!/bin/bash
# rocprofv3 evidence for profiles/: kernel-trace stats (graph mode, as benched), then HBM byte
# counters in separate PMC passes (eager mode so every dispatch is attributed).
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
prof() { local t=$1; shift; local tag=$1; shift
  timeout -k 10 "$t" rocprofv3 "$@" > "gpurun_out/$tag.log" 2>&1; local rc=$?; echo "$tag rc=$rc"; return $rc; }
for c in c2 c3 c4 c5; do
  prof 240 stats_$c --kernel-trace --stats -d gpurun_out/stats_$c -o run --output-format csv -- python3 bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline || exit 1
done
for c in c2 c3 c5; do
  prof 240 fetch_$c --pmc FETCH_SIZE -d gpurun_out/fetch_$c -o run --output-format csv -- python3 bench.py --config $c --eager --steps 4 --warmup 1 --no-cpu-baseline || exit 1
  prof 240 write_$c --pmc WRITE_SIZE -d gpurun_out/write_$c -o run --output-format csv -- python3 bench.py --config $c --eager --steps 4 --warmup 1 --no-cpu-baseline || exit 1
done
timeout -k 10 400 python3 bench.py > gpurun_out/bench_default.log 2>&1; echo "bench default rc=$?"
exit 0
