#!/bin/bash
# A/B of env switches on one bench_configs.py configuration: CFG=cfg5 AB="-|X=1" bash tools/ab_cfg.sh
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread $TESTS > gpurun_out/t.log 2>&1
  rc=$?; tail -1 gpurun_out/t.log; [ $rc -eq 0 ] || exit $rc
fi
IFS='|' read -ra ARMS <<< "${AB:--}"
for rep in ${REPS:-1 2}; do
  for arm in "${ARMS[@]}"; do
    [ "$arm" = "-" ] && arm=""
    env $arm timeout -k 10 300 python tools/bench_configs.py --only ${CFG:-cfg5} --steps ${STEPS:-6} --warmup 2 > gpurun_out/abc.json 2> gpurun_out/abc.err || { tail -5 gpurun_out/abc.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/abc.json').read().strip().splitlines()[-1]); print(sys.argv[1] or 'default', d['config'], d['value'], d['ms_per_step'])" "$arm"
  done
done
