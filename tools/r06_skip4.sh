#!/bin/bash
# timing-only: the step without the BN-backward statistics launches (wrong results), alternated with the default
set -u
cd "${GRAFT_REPO_ROOT:-.}"
VAR=HGNN_DIAG_SKIP_PART4 A=0 B=1 REPS=3 bash tools/ab.sh
