#!/bin/bash
# dA GEMM with 128-row tiles: GPU parity with HGNN_DA_BM=128, then alternating bench 64/128
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
[ "${SKIP_TESTS:-0}" = 1 ] || { HGNN_DA_BM=128 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/dabm_tests.log 2>&1; rc=$?; tail -3 gpurun_out/dabm_tests.log; [ $rc -ne 0 ] && exit $rc; }
VAR=HGNN_DA_BM A=64 B=128 REPS=${REPS:-4} bash tools/ab.sh
