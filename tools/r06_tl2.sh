#!/bin/bash
# current in-step timeline + per-wave stats of the headline step (stamp mode)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python tools/timeline.py --steps 6 > gpurun_out/timeline2.txt 2>&1 || { tail -5 gpurun_out/timeline2.txt; exit 1; }
timeout -k 10 300 python tools/wave_stats.py --steps 3 > gpurun_out/wave_stats2.txt 2>&1 || { tail -5 gpurun_out/wave_stats2.txt; exit 1; }
tail -3 gpurun_out/wave_stats2.txt
