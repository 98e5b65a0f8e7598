#!/bin/bash
# side-stream priority vs the RCCL process group's streams (GPU_MAX_HW_QUEUES=4, the box default)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for p in 0 -1 1; do
  HGNN_SIDE_PRIO=$p timeout -k 10 400 python tools/dp_ab.py --steps 100 --reps 2 > gpurun_out/dp_ab_p$p.txt 2>&1 || { tail -5 gpurun_out/dp_ab_p$p.txt; exit 1; }
  echo "HGNN_SIDE_PRIO=$p"; grep -E "no_dp|layer_b|one_bucket " gpurun_out/dp_ab_p$p.txt
done
for p in 0 -1; do
  HGNN_SIDE_PRIO=$p timeout -k 10 300 python bench.py --cpu-baseline 0 --roofline 0 --fwd-line 0 > gpurun_out/bp.json 2>/dev/null || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/bp.json').read().strip().splitlines()[-1]); print('plain bench prio=$p', d['value'], d['ms_per_step'])"
done
