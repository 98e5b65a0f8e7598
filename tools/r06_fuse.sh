#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_net.py tests/test_gpu_fullsize.py tests/test_gpu_train.py tests/test_gpu_switches.py tests/test_gpu_dp.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t.log 2>&1
rc=$?; tail -3 gpurun_out/t.log; [ $rc -eq 0 ] || exit $rc
SKIP_TESTS=1 CONFIGS="HGNN_BN_TAB=0;HGNN_BN_FUSE_DA=0;HGNN_BN_FUSE_DA=1" REPS=4 STEPS=100 bash tools/ab3.sh
