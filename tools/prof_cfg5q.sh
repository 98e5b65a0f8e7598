#!/bin/bash
# Kernel traces of the QM9-size CCN-2D configurations on the small-graph kernels: the per-graph drop-in
# (cfg5q_pergraph) and the batched step (cfg5q); outputs under gpurun_out/.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_c5qp -o run -- \
    python3 tools/bench_configs.py --only cfg5q_pergraph --steps 2 --warmup 1 > gpurun_out/c5qp_prof.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_c5q -o run -- \
    python3 tools/bench_configs.py --only cfg5q --steps 10 --warmup 3 > gpurun_out/c5q_prof.jsonl
python3 tools/kstats.py gpurun_out/kt_c5qp > gpurun_out/c5qp_kernel_stats.txt
python3 tools/kstats.py gpurun_out/kt_c5q > gpurun_out/c5q_kernel_stats.txt
