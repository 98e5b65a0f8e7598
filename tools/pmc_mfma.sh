#!/bin/bash
# MFMA utilisation of every GEMM of the bench step (SURVEY.md §8 d): one rocprofv3 PMC pass with
# SQ_VALU_MFMA_BUSY_CYCLES (MFMA pipe busy cycles summed over the SIMDs), SQ_BUSY_CYCLES, SQ_WAVES and
# GRBM_GUI_ACTIVE (GPU-active cycles summed over the 8 XCDs), kernel trace only, no other tracing.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE --kernel-trace \
    --output-format csv -d gpurun_out/pmc_mfma -o run \
    -- python3 bench.py --steps 3 --warmup 2 --cpu-baseline 0 --roofline 0 --fwd-line 0 > gpurun_out/pmc_mfma.log 2>&1
rc=$?; echo "pmc mfma rc=$rc"; tail -2 gpurun_out/pmc_mfma.log; [ $rc -eq 0 ] || exit $rc
python3 tools/pmc_mfma_summary.py gpurun_out/pmc_mfma > gpurun_out/pmc_mfma_summary.txt || exit $?
head -30 gpurun_out/pmc_mfma_summary.txt
