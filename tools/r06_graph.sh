#!/bin/bash
# eager vs HIP-graph replay of the whole step (bench.py --graph 1), alternating
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for r in 1 2 3; do
  for gmode in 0 1; do
    out=gpurun_out/graph_${gmode}_$r.json
    timeout -k 10 300 python bench.py --steps 100 --warmup 5 --cpu-baseline 0 --graph $gmode > $out 2> gpurun_out/graph.err || { tail -5 gpurun_out/graph.err; exit 1; }
    python -c "import json; d=json.loads(open('$out').read().strip().splitlines()[-1]); a=d.get('attribution') or {}; print('graph=$gmode', d['value'], d['ms_per_step'], d.get('launch'), 'host', a.get('host_enqueue_ms_per_step'), 'busy', a.get('gpu_busy_ms_per_step'), 'span', a.get('gpu_span_ms_per_step'))"
  done
done
