#!/bin/bash
# Round 3: CCN-2D config 5 kernel stats and per-kernel HBM traffic.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=6 bash tools/prof_cfg.sh cfg5 > gpurun_out/kt_cfg5_summary.txt || exit $?
head -20 gpurun_out/kt_cfg5_summary.txt
for P in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 200 rocprofv3 --pmc $P --kernel-trace --output-format csv -d gpurun_out/pmc_cfg5_$P -o run \
      -- python3 tools/bench_configs.py --only cfg5 --steps 4 --warmup 2 > gpurun_out/pmc_cfg5_$P.log 2>&1 || exit $?
done
python3 tools/pmc_summary.py gpurun_out/pmc_cfg5_FETCH_SIZE gpurun_out/pmc_cfg5_WRITE_SIZE gpurun_out/pmc_cfg5_traffic.json \
    > gpurun_out/pmc_cfg5_summary.txt || exit $?
head -20 gpurun_out/pmc_cfg5_summary.txt
