#!/bin/bash
# env sweep of the side stream's grid knobs with the round-6 kernels, each setting beside the default, two rounds
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
one() {
  local label=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 50 --warmup 5 --cpu-baseline 0 --roofline 0 --fwd-line 0 > gpurun_out/sw.json 2> gpurun_out/sw.err || { echo "$label FAILED"; tail -3 gpurun_out/sw.err; return 0; }
  python -c "import json; d=json.loads(open('gpurun_out/sw.json').read().strip().splitlines()[-1]); a=d.get('attribution') or {}; print('$label', d['ms_per_step'], 'host', a.get('host_enqueue_ms_per_step'), 'busy', a.get('gpu_busy_ms_per_step'))"
}
for r in 1 2; do
  one default X=1
  one dw_blocks_192 HGNN_DW_BLOCKS=192
  one dw_blocks_320 HGNN_DW_BLOCKS=320
  one default X=1
  one dw_ring_3 HGNN_DW_RING=3
  one dwd_grid_128 HGNN_DWD_GRID=128
  one dwd_grid_384 HGNN_DWD_GRID=384
done
