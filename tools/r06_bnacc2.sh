#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_net.py tests/test_gpu_fullsize.py tests/test_gpu_train.py -x -q --timeout 250 --timeout-method thread > gpurun_out/t.log 2>&1
rc=$?; tail -3 gpurun_out/t.log; [ $rc -eq 0 ] || exit $rc
VAR=HGNN_BN_ACC A=0 B=1 REPS=6 STEPS=100 bash tools/ab.sh || exit $?
