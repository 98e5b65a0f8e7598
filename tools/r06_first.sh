#!/bin/bash
# Round 6, first box: GPU suite, default bench twice (no CPU baseline), the forced RCCL world-1 bench and its
# kernel trace.  Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t.log 2>&1
rc=$?; tail -3 gpurun_out/t.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py --cpu-baseline 0 > gpurun_out/b$i.json 2> gpurun_out/b.err || { tail -5 gpurun_out/b.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/b$i.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['settle_steps'], d['attribution'])"
done
timeout -k 10 300 python bench.py --cpu-baseline 0 --roofline 0 --fwd-line 0 --force-dp 1 > gpurun_out/bdp.json 2> gpurun_out/bdp.err || { tail -5 gpurun_out/bdp.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/bdp.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['config'], d['comm'])"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_dp -o run -- python3 $GRAFT_REPO_ROOT/bench.py --cpu-baseline 0 --roofline 0 --fwd-line 0 --attribution 0 --force-dp 1 --settle-s 0.3 > $GRAFT_REPO_ROOT/gpurun_out/prof_dp.log 2>&1
rc=$?; echo "rocprof rc=$rc"; exit $rc
