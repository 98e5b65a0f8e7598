#!/bin/bash
# whole-step HIP-graph replay under the HIP runtime's graph-execution switches, against eager
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
run() {  # label, env..., then bench args after --
  local label=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python bench.py --steps 100 --warmup 5 --cpu-baseline 0 --roofline 0 --fwd-line 0 "$@" > gpurun_out/gq.json 2> gpurun_out/gq.err || { echo "$label FAILED"; tail -3 gpurun_out/gq.err; return 0; }
  python -c "import json; d=json.loads(open('gpurun_out/gq.json').read().strip().splitlines()[-1]); a=d.get('attribution') or {}; print('$label', d['ms_per_step'], d.get('launch'), 'host', a.get('host_enqueue_ms_per_step'))"
}
for r in 1 2; do
  run eager X=1 -- --graph 0
  run graph X=1 -- --graph 1
  run graph_nopkt DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 -- --graph 1
  run graph_q4 DEBUG_HIP_FORCE_GRAPH_QUEUES=4 -- --graph 1
  run graph_nopkt_q4 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 DEBUG_HIP_FORCE_GRAPH_QUEUES=4 -- --graph 1
done
