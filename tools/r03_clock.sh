#!/bin/bash
# Round 3: in-kernel clock of the GEMMs (diagnostic build), GRBM_GUI_ACTIVE effective clock, the
# per-graph CCN driver step (cfg3_pergraph) and its kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
HGNN_LIB_PATH=hgnn-2_amd/hgnn_amd/libhgnn_amd_clk.so timeout -k 10 180 python3 tools/clock_diag.py --settle-s 3 \
    > gpurun_out/clock_diag.json 2> gpurun_out/clock_diag.err || { tail -5 gpurun_out/clock_diag.err; exit 1; }
cat gpurun_out/clock_diag.json
timeout -k 10 200 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmc_grbm -o run \
    -- python3 bench.py --steps 3 --warmup 2 --cpu-baseline 0 --roofline 0 --fwd-line 0 > gpurun_out/pmc_grbm.log 2>&1 \
    || { tail -5 gpurun_out/pmc_grbm.log; exit 1; }
python3 tools/grbm_clock.py gpurun_out/pmc_grbm gemm > gpurun_out/grbm_clock.txt; cat gpurun_out/grbm_clock.txt
timeout -k 10 300 python3 tools/bench_configs.py --only cfg3_pergraph,cfg3,cfg3g > gpurun_out/cfg3pg.jsonl 2>&1 \
    || { tail -5 gpurun_out/cfg3pg.jsonl; exit 1; }
cat gpurun_out/cfg3pg.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_cfg3pg -o run \
    -- python3 tools/bench_configs.py --only cfg3_pergraph --steps 5 --warmup 1 > gpurun_out/prof_cfg3pg.log 2>&1 \
    || { tail -5 gpurun_out/prof_cfg3pg.log; exit 1; }
find gpurun_out/prof_cfg3pg -name "*kernel_stats.csv" | head -1 | xargs head -30
