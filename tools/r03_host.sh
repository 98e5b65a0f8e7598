#!/bin/bash
# Host-side profile of the per-graph CCN step, then the bench's roofline leg (dominant class timed alone).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/host_profile_ccn.py > gpurun_out/host_ccn.txt 2>&1 || { tail -20 gpurun_out/host_ccn.txt; exit 1; }
head -3 gpurun_out/host_ccn.txt
timeout -k 10 300 python3 bench.py --cpu-baseline 0 --fwd-line 0 > gpurun_out/bench_roof.json 2> gpurun_out/bench_roof.err || { tail -5 gpurun_out/bench_roof.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/bench_roof.json').read().strip().splitlines()[-1])
r=d['roofline']; print(d['value'], d['ms_per_step'], r['frac'], r['avg_launch_us'], {k: v['avg_launch_us'] for k, v in d['roofline_hbm'].items()})"
