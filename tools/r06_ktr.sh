#!/bin/bash
# kernel trace -> profiles/kernel_trace.json, then a bench line that reads it (frac_trace cross-check)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
SKIP_PMC=1 bash tools/prof_fused.sh > /dev/null || exit $?
cp gpurun_out/kernel_trace.json profiles/kernel_trace.json || exit $?
timeout -k 10 300 python bench.py --cpu-baseline 0 > gpurun_out/bench_ktr.json 2> gpurun_out/bench_ktr.err || { tail -5 gpurun_out/bench_ktr.err; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/bench_ktr.json').read().strip().splitlines()[-1]); r=d['roofline']
print(d['ms_per_step'], {k: r.get(k) for k in ('kernel','frac','avg_launch_us','trace_avg_launch_us','frac_trace')})
for k, v in d['roofline_hbm'].items(): print(k, {x: v.get(x) for x in ('frac','avg_launch_us','trace_avg_launch_us','frac_trace')})"
find gpurun_out -mindepth 1 -maxdepth 1 -type d -exec rm -rf {} +
