#!/bin/bash
# Round 3 checkpoint: the whole GPU suite, smoke, then the default bench (CPU baseline + parity leg).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_all.log 2>&1
rc=$?; tail -2 gpurun_out/t_all.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; tail -1 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_default.err; exit $rc; }
python3 -c "
import json; d=json.loads(open('gpurun_out/bench_default.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], 'roof', d['roofline']['frac'], d['roofline']['avg_launch_us'])
print('cpu', {k: d['cpu_baseline'][k] for k in ('value','cores','forward_s_median','backward_s_median','full_batch_step')})
print('parity', d['parity'])"
