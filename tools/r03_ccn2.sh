#!/bin/bash
# CCN-2D rework check: the CCN GPU tests, then config 5 (cfg3 for the CCN-1D regression) with kernel stats and PMC traffic.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_ccn.py tests/test_gpu_graph.py -x -v --timeout 200 --timeout-method thread > gpurun_out/t_ccn.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|error" gpurun_out/t_ccn.log | tail -25; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/bench_configs.py --only cfg5,cfg3 > gpurun_out/cfg5.jsonl 2> gpurun_out/cfg5.err || { tail -5 gpurun_out/cfg5.err; exit 1; }
cut -c1-300 gpurun_out/cfg5.jsonl
bash tools/r03_cfg5.sh
