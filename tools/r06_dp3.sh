#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for r in 1 2 3; do
for q in 8 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python bench.py --cpu-baseline 0 --roofline 0 --fwd-line 0 --force-dp 1 > gpurun_out/bdq.json 2> gpurun_out/bdq.err || { tail -5 gpurun_out/bdq.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/bdq.json').read().strip().splitlines()[-1]); a=d['attribution']; print('q=$q', d['value'], d['ms_per_step'], d['hw_queues'], 'host', a['host_enqueue_ms_per_step'], 'busy', a['gpu_busy_ms_per_step'], 'settle', a['settle_sample_ms_per_step'], d['comm']['allreduce_exposed_ms'])"
done
done
