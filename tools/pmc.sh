#!/bin/bash
# HBM traffic of every kernel of the bench step from rocprofv3 PMC counters.
# Two separate passes (FETCH_SIZE and WRITE_SIZE do not fit one TCC pass on
# gfx950; MI355X_MICROARCH.md "rocprofv3 PMC slots"), kernel trace only -- never
# combined with sys/runtime tracing.  Summarised by tools/pmc_summary.py.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 400 rocprofv3 --pmc $C --kernel-trace --output-format csv -d gpurun_out/pmc_$C -o run \
      -- python3 bench.py --steps 3 --warmup 2 --settle-s 0 --attribution 0 --cpu-baseline 0 --roofline 0 > gpurun_out/pmc_$C.log 2>&1
  rc=$?; echo "pmc $C rc=$rc"; tail -2 gpurun_out/pmc_$C.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
python3 tools/pmc_summary.py gpurun_out/pmc_FETCH_SIZE gpurun_out/pmc_WRITE_SIZE gpurun_out/pmc_traffic.json > gpurun_out/pmc_summary.txt
cat gpurun_out/pmc_summary.txt | head -40
