#!/bin/bash
# CCN small-graph path round 2: CCN + graph tests, kernel traces of cfg3 / per-graph, the CCN-1D configurations.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ccn.py tests/test_gpu_graph.py -x -v --timeout 120 --timeout-method thread > gpurun_out/t_small.log 2>&1
rc=$?; grep -E "FAIL|ERROR|passed|failed|Error" gpurun_out/t_small.log | tail -20; [ $rc -eq 0 ] || exit $rc
STEPS=6 bash tools/prof_cfg.sh cfg3 > gpurun_out/kt_cfg3s.txt || exit 1
head -8 gpurun_out/kt_cfg3s.txt
STEPS=2 bash tools/prof_cfg.sh cfg3_pergraph > gpurun_out/kt_pg.txt || exit 1
head -6 gpurun_out/kt_pg.txt
timeout -k 10 300 python3 tools/bench_configs.py --only cfg3,cfg3g,cfg3_pergraph > gpurun_out/cfg3_small.jsonl 2> gpurun_out/cfg3_small.err || { tail -5 gpurun_out/cfg3_small.err; exit 1; }
cut -c1-200 gpurun_out/cfg3_small.jsonl
