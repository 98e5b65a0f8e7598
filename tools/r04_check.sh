#!/bin/bash
# Round 4 check: the new GPU tests, the full GPU suite, bench --gpus 2 self-launch rehearsal (gloo on the
# one-GPU box), a default bench line.  Stops at the first crash / timeout.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    ${PYTEST_SEL:-} > gpurun_out/r04_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/r04_pytest.log; [ $rc -eq 0 ] || exit $rc
if [ "${SCALE2:-1}" = "1" ]; then
  HGNN_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 5 --warmup 2 --roofline 0 \
      --fwd-line 0 --settle-s 0.3 > gpurun_out/r04_gloo2.json 2> gpurun_out/r04_gloo2.err
  rc=$?; echo "gloo2 rc=$rc"; tail -c 600 gpurun_out/r04_gloo2.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/r04_gloo2.err; exit $rc; }
fi
if [ "${BENCH:-1}" = "1" ]; then
  timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > gpurun_out/r04_bench.json 2> gpurun_out/r04_bench.err
  rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/r04_bench.err; exit $rc; }
  python -c "
import json; d=json.loads(open('gpurun_out/r04_bench.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'], d['parity'] and d['parity']['pass'])
print(d['roofline']['class_ms_per_step_profile'])"
fi
