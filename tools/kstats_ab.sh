#!/bin/bash
# Kernel stats of the default bench under two settings of one switch: VAR=HGNN_X bash tools/kstats_ab.sh
set -euo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd /tmp && export TMPDIR=/tmp
for v in 0 1; do
    cd "$R"
    env ${VAR}=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/kt_ab_$v" -o run -- \
        python3 bench.py --steps 20 --warmup 5 --cpu-baseline 0 --roofline 0 --fwd-line 0 > "$R/gpurun_out/ab_$v.json"
    python3 "$R/tools/kstats.py" "$R/gpurun_out/kt_ab_$v" 22 > "$R/gpurun_out/kstats_ab_$v.txt"
done
