#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for m in 0 1 0 1; do
  timeout -k 10 300 python bench.py --cpu-baseline 0 --roofline 0 --fwd-line 0 --force-dp 1 --dp-single $m > gpurun_out/bdp$m.json 2> gpurun_out/bdp.err || { tail -5 gpurun_out/bdp.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/bdp$m.json').read().strip().splitlines()[-1]); print('single=$m', d['value'], d['ms_per_step'], d['hw_queues'], d['attribution']['host_enqueue_ms_per_step'], d['comm'] and d['comm']['allreduce_exposed_ms'])"
done
timeout -k 10 300 python bench.py --cpu-baseline 0 --roofline 0 --fwd-line 0 > gpurun_out/bp.json 2> gpurun_out/bp.err || { tail -5 gpurun_out/bp.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/bp.json').read().strip().splitlines()[-1]); print('plain', d['value'], d['ms_per_step'], d['hw_queues'])"
HGNN_BENCH_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --cpu-baseline 0 --roofline 0 --fwd-line 0 --steps 10 > gpurun_out/bg2.json 2> gpurun_out/bg2.err || { tail -5 gpurun_out/bg2.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/bg2.json').read().strip().splitlines()[-1]); print('gloo x2', d['value'], d['ms_per_step'], d['n_gpus'], d['hw_queues'], d['rank_ms_per_step'])"
