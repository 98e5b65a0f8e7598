#!/bin/bash
# Round-4 iteration: GPU tests (PYTEST_SEL narrows them), then the kernel trace of the bench step and a
# short bench line (no CPU baseline).  Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_SEL:-} \
      > gpurun_out/it_pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/it_pytest.log; [ $rc -eq 0 ] || exit $rc
fi
SKIP_PMC=1 bash tools/prof_fused.sh > /dev/null || exit $?
head -32 gpurun_out/kt_step.txt
timeout -k 10 300 python bench.py --cpu-baseline 0 --fwd-line 0 > gpurun_out/it_bench.json 2> gpurun_out/it_bench.err || { tail -5 gpurun_out/it_bench.err; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/it_bench.json').read().strip().splitlines()[-1])
print('bench', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'], {k: (v['avg_launch_us'], v['frac']) for k, v in d['roofline_hbm'].items()})"
