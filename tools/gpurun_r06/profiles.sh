#!/bin/bash
# Round-6 evidence: the GPU suite, the default bench line (with the CPU baseline), then rocprofv3
# on graph-replayed steps: kernel-trace stats, FETCH_SIZE / WRITE_SIZE passes per config (each its
# own run), the C3 / C5 calibration runs and the SQ counters of the C2 / C5 (VALU) and C3 (MFMA)
# kernels. Summarised by `python profiles/summarize.py r06`.
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fatal() { [ "$1" -eq 124 ] || [ "$1" -eq 137 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
prof() { local t=$1; shift; local tag=$1; shift
  timeout -s KILL "$t" rocprofv3 "$@" > "gpurun_out/$tag.log" 2>&1; local rc=$?; echo "$tag rc=$rc"
  if fatal $rc; then exit $rc; fi; return $rc; }
if [ "${SKIP_TESTS:-0}" != 1 ]; then
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06_final_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 gpurun_out/r06_final_tests.log
[ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 500 python3 -u bench.py > gpurun_out/r06_final_bench.json 2> gpurun_out/r06_final_bench.err; rc=$?
echo "bench rc=$rc"; fatal $rc && exit $rc
B="python3 bench.py --no-cpu-baseline --no-other-configs --steps 48 --warmup 3 --warm-ms 20"
for c in c2 c3 c4 c5; do
  rm -rf gpurun_out/stats_$c
  prof 240 stats_$c --kernel-trace --stats -d gpurun_out/stats_$c -o run --output-format csv -- $B --config $c || exit 1
done
P="python3 bench.py --no-cpu-baseline --no-other-configs --steps 16 --warmup 2 --warm-ms 0"
for c in c2 c3 c4 c5; do
  rm -rf gpurun_out/fetch_$c gpurun_out/write_$c
  prof 150 fetch_$c --pmc FETCH_SIZE -d gpurun_out/fetch_$c -o run --output-format csv -- $P --config $c || exit 1
  prof 150 write_$c --pmc WRITE_SIZE -d gpurun_out/write_$c -o run --output-format csv -- $P --config $c || exit 1
done
rm -rf gpurun_out/fetch_c3cal gpurun_out/fetch_c5cal gpurun_out/write_c5cal
prof 150 fetch_c3cal --pmc FETCH_SIZE -d gpurun_out/fetch_c3cal -o run --output-format csv -- $P --config c3 --particles-per-gpu 32 || exit 1
prof 150 fetch_c5cal --pmc FETCH_SIZE -d gpurun_out/fetch_c5cal -o run --output-format csv -- $P --config c5 --particles-per-gpu 64 || exit 1
prof 150 write_c5cal --pmc WRITE_SIZE -d gpurun_out/write_c5cal -o run --output-format csv -- $P --config c5 --particles-per-gpu 64 || exit 1
rm -rf gpurun_out/wait_c5 gpurun_out/vtype_c5 gpurun_out/wait_c2 gpurun_out/vtype_c2 gpurun_out/wait_c3 gpurun_out/vtype_c3
prof 150 wait_c5 --kernel-include-regex mi_site_program --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -d gpurun_out/wait_c5 -o run --output-format csv -- $P --config c5 || exit 1
prof 150 vtype_c5 --kernel-include-regex mi_site_program --pmc SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM GRBM_GUI_ACTIVE -d gpurun_out/vtype_c5 -o run --output-format csv -- $P --config c5 || exit 1
prof 150 wait_c2 --kernel-include-regex k_site_bcast --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE -d gpurun_out/wait_c2 -o run --output-format csv -- $P --config c2 || exit 1
prof 150 vtype_c2 --kernel-include-regex k_site_bcast --pmc SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_SALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE -d gpurun_out/vtype_c2 -o run --output-format csv -- $P --config c2 || exit 1
prof 150 wait_c3 --kernel-include-regex k_linear --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA GRBM_GUI_ACTIVE -d gpurun_out/wait_c3 -o run --output-format csv -- $P --config c3 || exit 1
prof 150 vtype_c3 --kernel-include-regex k_linear --pmc SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_SMEM GRBM_GUI_ACTIVE -d gpurun_out/vtype_c3 -o run --output-format csv -- $P --config c3 || exit 1
exit 0
