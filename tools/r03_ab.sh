#!/bin/bash
# A/B of environment switches + the step's kernel trace (generic driver for round 3).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "${AB1:-}" ]; then AB="$AB1" REPS="${REPS:-1 2}" bash tools/ab_env.sh || exit 1; fi
if [ "${TRACE:-1}" = "1" ]; then SKIP_PMC=1 bash tools/prof_fused.sh | head -${TRACE_LINES:-25} || exit 1; fi
