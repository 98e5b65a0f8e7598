#!/bin/bash
# GPU tests + two short benches (no CPU baseline); prints value, ms/step and the class profile.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t.log 2>&1
rc=$?; tail -3 gpurun_out/t.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py --cpu-baseline 0 ${BENCH_ARGS:-} > gpurun_out/b$i.json 2> gpurun_out/b.err || { tail -5 gpurun_out/b.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/b$i.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['class_ms_per_step_profile'])"
done
