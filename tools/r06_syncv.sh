#!/bin/bash
# stream value syncs for the backward's forks / joins: GPU parity with HGNN_SYNC_VALUE=1, then alternating bench 0/1
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
[ "${SKIP_TESTS:-0}" = 1 ] || { HGNN_SYNC_VALUE=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/syncv_tests.log 2>&1; rc=$?; tail -3 gpurun_out/syncv_tests.log; [ $rc -ne 0 ] && exit $rc; }
VAR=HGNN_SYNC_VALUE A=0 B=1 REPS=${REPS:-4} bash tools/ab.sh
