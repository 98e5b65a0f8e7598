#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python tools/dp_host_prof.py --steps 200 > gpurun_out/dph_layer.txt 2>&1 || { tail -5 gpurun_out/dph_layer.txt; exit 1; }
head -4 gpurun_out/dph_layer.txt | grep dp=
timeout -k 10 300 python tools/dp_host_prof.py --steps 200 --single 1 > gpurun_out/dph_single.txt 2>&1 || { tail -5 gpurun_out/dph_single.txt; exit 1; }
grep "dp=" gpurun_out/dph_single.txt
for m in 0 1; do
timeout -k 10 300 python bench.py --cpu-baseline 0 --roofline 0 --fwd-line 0 --force-dp 1 --dp-single $m > gpurun_out/bdp$m.json 2> gpurun_out/bdp.err || { tail -5 gpurun_out/bdp.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/bdp$m.json').read().strip().splitlines()[-1]); print('single=$m', d['value'], d['ms_per_step'], d['comm'], d['attribution']['host_enqueue_ms_per_step'], d['attribution']['gpu_busy_ms_per_step'])"
done
