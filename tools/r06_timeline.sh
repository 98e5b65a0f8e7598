#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python tools/timeline.py --steps 6 --json gpurun_out/tl.json > gpurun_out/timeline.txt 2>&1 || { tail -5 gpurun_out/timeline.txt; exit 1; }
tail -40 gpurun_out/timeline.txt
