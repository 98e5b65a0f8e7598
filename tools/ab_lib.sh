#!/bin/bash
# Alternating A/B of two builds of the library on the headline bench: LIBS="path_a|path_b" (HGNN_LIB_PATH;
# "in-tree" = the in-tree library; bash's read drops a trailing empty field), REPS=3.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
IFS='|' read -ra L <<< "${LIBS}"
for rep in $(seq 1 ${REPS:-3}); do
  for lib in "${L[@]}"; do
    [ "$lib" = in-tree ] && lib=
    HGNN_LIB_PATH=$lib timeout -k 10 300 python bench.py --cpu-baseline 0 --roofline 0 --fwd-line 0 --steps ${STEPS:-50} \
        > gpurun_out/ab_lib.json 2> gpurun_out/ab_lib.err || { tail -5 gpurun_out/ab_lib.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab_lib.json').read().strip().splitlines()[-1]); print('%-50s'%(sys.argv[1] or 'in-tree'), d['value'], d['ms_per_step'], flush=True)" "$lib"
  done
done
