#!/bin/bash
# One rocprofv3 PMC pass of wave-state counters (SQ block, 8 slots) over a short bench run;
# per-kernel sums by tools/pmc_sq_summary.py.  Kernel trace only, no other tracing.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
C="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD"
timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d gpurun_out/pmc_sq -o run \
    -- python3 bench.py --steps 3 --warmup 2 --cpu-baseline 0 --roofline 0 > gpurun_out/pmc_sq.log 2>&1
rc=$?; echo "pmc sq rc=$rc"; tail -2 gpurun_out/pmc_sq.log
[ $rc -eq 0 ] || exit $rc
python3 tools/pmc_sq_summary.py gpurun_out/pmc_sq > gpurun_out/pmc_sq_summary.txt
cat gpurun_out/pmc_sq_summary.txt | head -30
