#!/bin/bash
# Round 3: net GPU tests, then configs cfg4 / cfg1g / cfg2 (A/B arms in AB) and the default bench.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_net.py tests/test_gpu_ops.py tests/test_gpu_fullsize.py tests/test_gpu_train.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_cfg.log 2>&1
rc=$?; tail -1 gpurun_out/t_cfg.log; [ $rc -eq 0 ] || exit $rc
for c in ${CFGS:-cfg4 cfg1g}; do CFG=$c REPS="${REPS:-1 2}" bash tools/ab_cfg.sh || exit 1; done
AB="${AB2:-|}" REPS="1 2" bash tools/ab_env.sh
