#!/bin/bash
# Round 3: kernel trace of the headline step, A/B of the dW block target, side stream vs graph replay.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
SKIP_PMC=1 bash tools/prof_fused.sh || exit $?
AB="HGNN_DW_BLOCKS=128|HGNN_DW_BLOCKS=192|HGNN_DW_BLOCKS=256" REPS="1 2" bash tools/ab_env.sh || exit 1
AB="HGNN_SIDE=0|" REPS="1" bash tools/ab_env.sh || exit 1
AB="HGNN_SIDE=0|" REPS="1" BENCH_ARGS="--graph 1" bash tools/ab_env.sh || exit 1
