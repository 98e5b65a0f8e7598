#!/bin/bash
# Round-end style measurement: GPU tests, smoke, bench (+ CPU baseline), rocprof kernel stats,
# PMC HBM traffic passes and the other BASELINE configs.  Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
bash tools/gpu_check.sh || exit $?
bash tools/pmc.sh || exit $?
timeout -k 10 600 python tools/bench_configs.py > gpurun_out/configs.jsonl 2> gpurun_out/configs.err
rc=$?; echo "configs rc=$rc"; cat gpurun_out/configs.jsonl | cut -c1-200
exit $rc
