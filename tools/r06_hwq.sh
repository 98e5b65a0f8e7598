#!/bin/bash
# Does an initialised RCCL process group push the executor's side stream onto the main stream's hardware queue?
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for q in 4 8; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 400 python tools/dp_ab.py --steps 100 --reps 2 > gpurun_out/dp_ab_q$q.txt 2>&1 || { tail -5 gpurun_out/dp_ab_q$q.txt; exit 1; }
  echo "GPU_MAX_HW_QUEUES=$q"; grep -E "wall" gpurun_out/dp_ab_q$q.txt
done
