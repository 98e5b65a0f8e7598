#!/bin/bash
# Same-box A/B of config 1 (GNN_simple L=20, 32 SBM-50 graphs, eager and HIP-graph replay) between the
# round-2 final tree (a git worktree at _r2, built there) and this tree: alternating runs.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
for rep in 1 2 3; do
    for arm in r2 head; do
        if [ $arm = r2 ]; then dir=_r2; else dir=.; fi
        (cd $dir && timeout -k 10 200 python3 tools/bench_configs.py --only cfg1,cfg1g --steps 30 --warmup 5) \
            | sed "s/^/$arm /" >> gpurun_out/ab_cfg1.txt || { echo "$arm failed"; exit 1; }
    done
done
# kernel traces of both arms (launches per step)
cd /tmp && export TMPDIR=/tmp
for arm in r2 head; do
    if [ $arm = r2 ]; then dir=$R/_r2; else dir=$R; fi
    cd $dir
    timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/kt_cfg1_$arm -o run -- \
        python3 tools/bench_configs.py --only cfg1 --steps 20 --warmup 2 > /dev/null || { echo "trace $arm failed"; exit 1; }
    python3 $R/tools/kstats.py $R/gpurun_out/kt_cfg1_$arm 40 > $R/gpurun_out/cfg1_kstats_$arm.txt
done
