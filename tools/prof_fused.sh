#!/bin/bash
# Kernel trace (per-dispatch durations) + one SQ wave-state PMC pass of a short bench run.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt -o run \
    -- python3 bench.py --steps 5 --warmup 2 --settle-s 0 --attribution 0 --cpu-baseline 0 --roofline 0 --fwd-line 0 > gpurun_out/kt.log 2>&1
rc=$?; echo "kt rc=$rc"; [ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/kt -name "*kernel_trace.csv" | head -1); python3 tools/trace_step.py "$f" 7 gpurun_out/kernel_trace.json > gpurun_out/kt_step.txt 2>&1; head -45 gpurun_out/kt_step.txt
[ "${SKIP_PMC:-0}" = "1" ] && exit 0
C="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS"
timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d gpurun_out/pmc_sq -o run \
    -- python3 bench.py --steps 3 --warmup 2 --settle-s 0 --attribution 0 --cpu-baseline 0 --roofline 0 --fwd-line 0 > gpurun_out/pmc_sq.log 2>&1
rc=$?; echo "pmc sq rc=$rc"; tail -2 gpurun_out/pmc_sq.log
[ $rc -eq 0 ] || exit $rc
python3 tools/pmc_sq_summary.py gpurun_out/pmc_sq > gpurun_out/pmc_sq_summary.txt
cat gpurun_out/pmc_sq_summary.txt | head -30
