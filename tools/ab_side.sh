#!/bin/bash
# A/B of env switches (AB="arm1|arm2", "-" = default) on the headline bench, alternating runs;
# optional GPU test selection first (TESTS="-k expr").
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread $TESTS > gpurun_out/t.log 2>&1
  rc=$?; tail -3 gpurun_out/t.log; [ $rc -eq 0 ] || exit $rc
fi
IFS='|' read -ra ARMS <<< "${AB:--}"
for rep in ${REPS:-1 2 3}; do
  for arm in "${ARMS[@]}"; do
    [ "$arm" = "-" ] && arm=""
    env $arm timeout -k 10 300 python bench.py --cpu-baseline 0 --roofline 0 --fwd-line 0 ${BENCH_ARGS:-} > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab.json').read().strip().splitlines()[-1]); print(sys.argv[1] or 'default', d['value'], d['ms_per_step'])" "$arm"
  done
done
