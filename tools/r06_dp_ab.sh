#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 500 python tools/dp_ab.py --steps 100 --reps 3 > gpurun_out/dp_ab.txt 2>&1 || { tail -5 gpurun_out/dp_ab.txt; exit 1; }
grep -E "wall" gpurun_out/dp_ab.txt
