#!/bin/bash
# A/B/C of env settings on one box: alternating bench runs (no CPU baseline), GPU tests first.
# usage: CONFIGS="HGNN_X=0;HGNN_X=1 HGNN_Y=2" REPS=2 bash tools/ab3.sh
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t.log 2>&1
  rc=$?; tail -2 gpurun_out/t.log; [ $rc -eq 0 ] || exit $rc
fi
IFS=';' read -ra CFG <<< "$CONFIGS"
for r in $(seq 1 ${REPS:-2}); do
  for c in "${CFG[@]}"; do
    out=gpurun_out/ab3.json
    env $c timeout -k 10 300 python bench.py --steps ${STEPS:-50} --warmup 5 --cpu-baseline 0 ${BENCH_ARGS:-} > $out 2> gpurun_out/ab.err
    rc=$?; if [ $rc -ne 0 ]; then tail -5 gpurun_out/ab.err; exit $rc; fi
    python -c "import json,sys; d=json.loads(open('$out').read().strip().splitlines()[-1]); p=d['roofline']['class_ms_per_step_profile']; print('%-28s'%sys.argv[1][-28:], d['value'], d['ms_per_step'], ' '.join('%s %.3f' % (k, p[k]) for k in ('struct','agg_fwd','gemm_fwd','bn_bwd','gemm_da','agg_bwd','gemm_dw')))" "$c"
  done
done
