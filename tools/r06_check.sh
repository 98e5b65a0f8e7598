#!/bin/bash
# GPU suite, smoke, two default bench lines (no CPU baseline), forced RCCL world-1 bench with layer buckets and one bucket
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t.log 2>&1
rc=$?; tail -3 gpurun_out/t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1 || exit 1
for i in 1 2; do
  timeout -k 10 300 python bench.py --cpu-baseline 0 > gpurun_out/b$i.json 2> gpurun_out/b.err || { tail -5 gpurun_out/b.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/b$i.json').read().strip().splitlines()[-1]); a=d['attribution']; print(d['value'], d['ms_per_step'], d['settle_steps'], a['host_enqueue_ms_per_step'], a['gpu_busy_ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'])"
done
for m in 0 1; do
  timeout -k 10 300 python bench.py --cpu-baseline 0 --roofline 0 --fwd-line 0 --force-dp 1 --dp-single $m > gpurun_out/bdp$m.json 2> gpurun_out/bdp.err || { tail -5 gpurun_out/bdp.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/bdp$m.json').read().strip().splitlines()[-1]); print('single=$m', d['value'], d['ms_per_step'], d['attribution']['host_enqueue_ms_per_step'], d['comm'])"
done
