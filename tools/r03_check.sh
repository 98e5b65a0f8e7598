#!/bin/bash
# Round 3 check of a change on the headline path: the net GPU tests, three default-shape benches
# (value, ms/step), then the kernel trace of one bench (per-kernel time per step).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_net.py tests/test_gpu_ops.py tests/test_gpu_fullsize.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_chk.log 2>&1
rc=$?; tail -2 gpurun_out/t_chk.log; [ $rc -eq 0 ] || exit $rc
AB="${AB:-|}" REPS="${REPS:-1 2 3}" bash tools/ab_env.sh || exit 1
SKIP_PMC=1 bash tools/prof_fused.sh | head -32
