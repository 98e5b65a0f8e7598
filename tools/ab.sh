#!/bin/bash
# A/B of an env switch on one box: alternating bench runs (no CPU baseline).
# usage: VAR=HGNN_FWD_BF3 A=0 B=1 REPS=3 bash tools/ab.sh
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for r in $(seq 1 ${REPS:-3}); do
  for v in ${A:-0} ${B:-1}; do
    out=gpurun_out/ab_$(basename "$v")_${r}.json
    env $VAR=$v timeout -k 10 300 python bench.py --steps ${STEPS:-50} --warmup 5 --cpu-baseline 0 ${BENCH_ARGS:-} > $out 2> gpurun_out/ab.err
    rc=$?; if [ $rc -ne 0 ]; then tail -5 gpurun_out/ab.err; exit $rc; fi
    python -c "import json; d=json.loads(open('$out').read().strip().splitlines()[-1]); a=d.get('attribution') or {}; print('$VAR=$v', d['value'], d['ms_per_step'], 'host', a.get('host_enqueue_ms_per_step'), 'busy', a.get('gpu_busy_ms_per_step'), 'span', a.get('gpu_span_ms_per_step'), d['roofline']['class_ms_per_step_profile'])"
  done
done
