#!/bin/bash
# Alternating A/B of environment arms on the headline bench (value and ms per step per run), optional GPU
# tests first.  AB="HGNN_X=0|HGNN_X=1|" (arms separated by |; an empty arm = defaults), REPS=3, TESTS="tests/test_gpu_net.py tests/test_gpu_fullsize.py"
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 500 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ab5_tests.log 2>&1
  rc=$?; tail -2 gpurun_out/ab5_tests.log; [ $rc -eq 0 ] || exit $rc
fi
IFS='|' read -ra ARMS <<< "${AB:-|}"
for rep in $(seq 1 ${REPS:-3}); do
  for arm in "${ARMS[@]}"; do
    env $arm timeout -k 10 300 python bench.py --cpu-baseline 0 --roofline 0 --fwd-line 0 --steps ${STEPS:-50} ${BENCH_ARGS:-} \
        > gpurun_out/ab5.json 2> gpurun_out/ab5.err || { tail -5 gpurun_out/ab5.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab5.json').read().strip().splitlines()[-1]); print('%-40s'%(sys.argv[1] or 'default'), d['value'], d['ms_per_step'], flush=True)" "$arm"
  done
done
