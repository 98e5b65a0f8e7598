#!/bin/bash
# Whole-step HIP-graph replay (bench.py --graph 1) vs eager under the HIP runtime's graph knobs (packet capture off, forced graph queues), headline bench, 50 steps
set -u
cd "${GRAFT_REPO_ROOT:-.}"
for arm in "eager|" "graph|" "graph|DEBUG_CLR_GRAPH_PACKET_CAPTURE=0" "graph|DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 DEBUG_HIP_FORCE_GRAPH_QUEUES=4"; do
  mode=${arm%%|*}; envs=${arm#*|}
  flag=""; [ "$mode" = graph ] && flag="--graph 1"
  env $envs timeout -k 10 300 python bench.py $flag --cpu-baseline 0 --roofline 0 --fwd-line 0 --steps 50 > gpurun_out/gx.json 2> gpurun_out/gx.err || { tail -3 gpurun_out/gx.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/gx.json').read().strip().splitlines()[-1]); print('%-70s'%sys.argv[1], d['value'], d['ms_per_step'], d.get('launch'))" "$arm"
done
