#!/bin/bash
# Quick GPU iteration: parity tests (stop at first failure), then a short bench without the CPU leg.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread ${PYTEST_ARGS:-} \
      ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/t.log 2>&1
  rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/t.log | tail -8; [ $rc -eq 0 ] || exit $rc
fi
[ "${SKIP_BENCH:-0}" = "1" ] && exit 0
for i in ${BENCH_RUNS:-1}; do
  timeout -k 10 300 python bench.py --cpu-baseline 0 ${BENCH_ARGS:-} > gpurun_out/b$i.json 2> gpurun_out/b.err || { tail -5 gpurun_out/b.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/b$i.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['class_ms_per_step_profile'], d['roofline_fwd']['ms_per_forward'])"
done
