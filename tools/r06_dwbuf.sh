#!/bin/bash
# dW ring with buffer loads: GPU parity, then alternating bench runs against the previous build (ab/libbase.so)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
[ "${SKIP_TESTS:-0}" = 1 ] || timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/dwbuf_tests.log 2>&1
rc=$?; [ "${SKIP_TESTS:-0}" = 1 ] || tail -3 gpurun_out/dwbuf_tests.log; [ $rc -ne 0 ] && exit $rc
VAR=HGNN_LIB_PATH A=$PWD/ab/libbase.so B=$PWD/hgnn-2_amd/hgnn_amd/libhgnn_amd.so REPS=${REPS:-4} bash tools/ab.sh
