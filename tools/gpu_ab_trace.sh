#!/bin/bash
# A/B of env switches (AB, see ab_side.sh) followed by a kernel trace of the default bench step.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
bash tools/ab_side.sh || exit $?
SKIP_PMC=1 bash tools/prof_fused.sh > /dev/null || exit $?
head -40 gpurun_out/kt_step.txt
