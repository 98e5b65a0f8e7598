#!/bin/bash
# A/B of environment switches on the headline bench: alternating runs, one line per run.
#   AB="HGNN_SERIAL_BWD=1|" bash tools/ab_env.sh    (arms separated by |, empty = default)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
IFS='|' read -ra ARMS <<< "${AB:-|}"
for rep in ${REPS:-1 2}; do
  for arm in "${ARMS[@]}"; do
    env $arm timeout -k 10 300 python bench.py --cpu-baseline 0 --roofline 0 --fwd-line 0 ${BENCH_ARGS:-} > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab.json').read().strip().splitlines()[-1]); print(sys.argv[1] or 'default', d['value'], d['ms_per_step'])" "$arm"
  done
done
