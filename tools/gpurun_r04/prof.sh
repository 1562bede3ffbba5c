#!/bin/bash
# rocprofv3 evidence for profiles/ (round tag r04): kernel-trace stats of graph-replay steps as
# benched, then separate PMC passes (FETCH_SIZE, WRITE_SIZE) on eager steps, and the C5 site
# program's FETCH_SIZE calibration (K = 64: one particle block, each element's inputs read once).
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fatal() { [ "$1" -eq 124 ] || [ "$1" -eq 137 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
prof() { local t=$1; shift; local tag=$1; shift
  timeout -s KILL "$t" rocprofv3 "$@" > "gpurun_out/$tag.log" 2>&1; local rc=$?; echo "$tag rc=$rc"
  if fatal $rc; then exit $rc; fi; return $rc; }
B="python3 bench.py --no-cpu-baseline --no-other-configs"
for c in ${CONFIGS:-c2 c3 c4 c5}; do
  prof 240 stats_$c --kernel-trace --stats -d gpurun_out/stats_$c -o run --output-format csv -- $B --config $c --steps 20 --warmup 3 || exit 1
done
[ "${STATS_ONLY:-0}" = 1 ] && exit 0
for c in c2 c4 c5; do
  prof 120 fetch_$c --pmc FETCH_SIZE -d gpurun_out/fetch_$c -o run --output-format csv -- $B --config $c --eager --steps 4 --warmup 1
  prof 120 write_$c --pmc WRITE_SIZE -d gpurun_out/write_$c -o run --output-format csv -- $B --config $c --eager --steps 4 --warmup 1
done
prof 120 fetch_c5cal --pmc FETCH_SIZE -d gpurun_out/fetch_c5cal -o run --output-format csv -- $B --config c5 --particles-per-gpu 64 --eager --steps 4 --warmup 1
prof 120 write_c5cal --pmc WRITE_SIZE -d gpurun_out/write_c5cal -o run --output-format csv -- $B --config c5 --particles-per-gpu 64 --eager --steps 4 --warmup 1
exit 0
