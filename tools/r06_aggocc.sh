#!/bin/bash
# agg_fwd occupancy: builds with amdgpu_waves_per_eu 7 / 8 on k_agg_fwd_rpw (ab/lib_w7.so, ab/lib_w8.so) vs in-tree
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for r in 1 2 3; do
  for v in hgnn-2_amd/hgnn_amd/libhgnn_amd.so ab/lib_w7.so ab/lib_w8.so; do
    out=gpurun_out/occ_$(basename $v)_$r.json
    HGNN_LIB_PATH=$PWD/$v timeout -k 10 300 python bench.py --steps 50 --warmup 5 --cpu-baseline 0 > $out 2> gpurun_out/occ.err || { tail -5 gpurun_out/occ.err; exit 1; }
    python -c "import json; d=json.loads(open('$out').read().strip().splitlines()[-1]); a=d.get('attribution') or {}; r=d['roofline_hbm']['agg_fwd']; print('$v', d['ms_per_step'], 'host', a.get('host_enqueue_ms_per_step'), 'agg_fwd us', r['avg_launch_us'], 'frac', r['frac'], d['roofline']['class_ms_per_step_profile'].get('agg_fwd'))"
  done
done
