#!/bin/bash
# Round-end measurement set: profile_round.sh (kernel trace/stats, PMC traffic, SQ wave states,
# CCN profiles, all configs), then the default bench line (CPU baseline + parity leg) reading the
# fresh PMC traffic.  Results under gpurun_out/ (copied into profiles/ by the caller).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
bash tools/profile_round.sh || exit $?
cp gpurun_out/pmc_traffic.json profiles/pmc_traffic.json || exit $?
cp gpurun_out/kernel_trace.json profiles/kernel_trace.json || exit $?
timeout -k 10 600 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -5 gpurun_out/bench_default.err; exit 1; }
tail -1 gpurun_out/bench_default.json | cut -c1-600
# the raw rocprofv3 directories stay on the box (gpurun merges back at most 64 MiB): summaries only
find gpurun_out -mindepth 1 -maxdepth 1 -type d -exec rm -rf {} +
