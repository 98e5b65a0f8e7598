#!/bin/bash
# Kernel trace of one tools/bench_configs.py configuration: CFG=cfg1g bash tools/prof_cfg.sh
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
CFG=${CFG:-cfg1g}
rm -rf gpurun_out/kt_$CFG
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_$CFG -o run \
    -- python3 tools/bench_configs.py --only $CFG --steps ${STEPS:-5} --warmup 2 > gpurun_out/kt_$CFG.log 2>&1
rc=$?; echo "kt rc=$rc"; tail -2 gpurun_out/kt_$CFG.log; exit $rc
