#!/bin/bash
# Same-box A/B of the CCN-1D small-graph path (HGNN_CCN_SMALL=0: general path) on the per-graph and
# batched CCN-1D configurations, alternating.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
: > gpurun_out/ab_small.jsonl
for rep in 1 2; do
  for sm in 0 1; do
    HGNN_CCN_SMALL=$sm timeout -k 10 200 python3 tools/bench_configs.py --only cfg3,cfg3_pergraph > gpurun_out/ab_small_$sm.jsonl 2> gpurun_out/ab_small.err || { tail -5 gpurun_out/ab_small.err; exit 1; }
    python3 -c "
import json,sys
for l in open('gpurun_out/ab_small_$sm.jsonl'):
    d=json.loads(l); d['small']=$sm; d['rep']=$rep; print(json.dumps(d))" >> gpurun_out/ab_small.jsonl
  done
done
python3 -c "
import json
for l in open('gpurun_out/ab_small.jsonl'):
    d=json.loads(l); print(d['rep'], 'small', d['small'], d['config'], d['ms_per_step'], d.get('ms_per_graph'))"
