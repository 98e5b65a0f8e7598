#!/bin/bash
# Round 3 A/B: GPU suite subset for the dW reduction, then alternating bench arms (AB, separated by |).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_net.py tests/test_gpu_train.py tests/test_gpu_graph.py tests/test_gpu_ccn.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_ab.log 2>&1
rc=$?; tail -2 gpurun_out/t_ab.log; [ $rc -eq 0 ] || exit $rc
AB="${AB:-|}" REPS="${REPS:-1 2 3}" bash tools/ab_env.sh
