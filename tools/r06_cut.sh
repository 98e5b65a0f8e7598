#!/bin/bash
# Round 6: diagonal I / D columns -- focused parity tests, the whole GPU suite, an alternating A/B of
# HGNN_DIAG_ID (0 = the full aggregate), and the forced RCCL world-1 bench after the DP host-path fix.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_switches.py tests/test_gpu_net.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t1.log 2>&1
rc=$?; tail -15 gpurun_out/t1.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t.log 2>&1
rc=$?; tail -3 gpurun_out/t.log; [ $rc -eq 0 ] || exit $rc
VAR=HGNN_DIAG_ID A=0 B=1 REPS=3 STEPS=100 bash tools/ab.sh || exit $?
timeout -k 10 300 python bench.py --cpu-baseline 0 --roofline 0 --fwd-line 0 --force-dp 1 > gpurun_out/bdp.json 2> gpurun_out/bdp.err || { tail -5 gpurun_out/bdp.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/bdp.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['comm'], d['attribution'])"
