#!/bin/bash
# aggregation block size: AGG_BLOCK_WAVES 2 / 8 builds (ab/lib_bw*.so) vs the in-tree 4
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for r in 1 2 3; do
  for v in hgnn-2_amd/hgnn_amd/libhgnn_amd.so ab/lib_bw2.so ab/lib_bw8.so; do
    out=gpurun_out/bw_$(basename $v)_$r.json
    HGNN_LIB_PATH=$PWD/$v timeout -k 10 300 python bench.py --steps 50 --warmup 5 --cpu-baseline 0 > $out 2> gpurun_out/bw.err || { tail -5 gpurun_out/bw.err; exit 1; }
    python -c "import json; d=json.loads(open('$out').read().strip().splitlines()[-1]); h=d['roofline_hbm']; print('$v', d['ms_per_step'], 'agg_fwd', h['agg_fwd']['avg_launch_us'], h['agg_fwd']['frac'], 'agg_bwd', h['agg_bwd']['avg_launch_us'], h['agg_bwd']['frac'])"
  done
done
