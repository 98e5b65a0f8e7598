#!/bin/bash
# CCN small-graph path: CCN + graph tests, the CCN-1D configurations, the per-graph host profile.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ccn.py tests/test_gpu_graph.py -x -v --timeout 120 --timeout-method thread > gpurun_out/t_small.log 2>&1
rc=$?; grep -E "FAIL|ERROR|passed|failed|Error" gpurun_out/t_small.log | tail -20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/bench_configs.py --only cfg3,cfg3g,cfg3_pergraph > gpurun_out/cfg3_small.jsonl 2> gpurun_out/cfg3_small.err || { tail -5 gpurun_out/cfg3_small.err; exit 1; }
cut -c1-200 gpurun_out/cfg3_small.jsonl
timeout -k 10 300 python3 -u tools/host_profile_ccn.py > gpurun_out/host_ccn_small.txt 2>&1 || { tail -20 gpurun_out/host_ccn_small.txt; exit 1; }
head -3 gpurun_out/host_ccn_small.txt
