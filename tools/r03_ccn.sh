#!/bin/bash
# Round 3: CCN GPU tests, then config-5 / config-3 timings and config-5 kernel stats + traffic.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_ccn.py tests/test_gpu_graph.py -x -q --timeout 200 --timeout-method thread > gpurun_out/tc.log 2>&1
rc=$?; tail -3 gpurun_out/tc.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/bench_configs.py --only cfg5,cfg3,cfg3g,cfg3_pergraph > gpurun_out/ccn_cfgs.jsonl 2>&1 || { tail -5 gpurun_out/ccn_cfgs.jsonl; exit 1; }
cut -c1-220 gpurun_out/ccn_cfgs.jsonl
bash tools/r03_cfg5.sh
