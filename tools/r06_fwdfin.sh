#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
HGNN_BN_TAB=0 HGNN_BN_FWD_FIN=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_net.py tests/test_gpu_fullsize.py tests/test_gpu_train.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t.log 2>&1
rc=$?; tail -3 gpurun_out/t.log; [ $rc -eq 0 ] || exit $rc
SKIP_TESTS=1 CONFIGS="HGNN_BN_TAB=0;HGNN_BN_TAB=0 HGNN_BN_FWD_FIN=1" REPS=5 STEPS=100 bash tools/ab3.sh
