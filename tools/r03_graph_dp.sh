#!/bin/bash
# Round 3: the HIP-graph capture hazard with the eager output kept as values only (DIAG_DETACH=1),
# bench.py --graph 1 vs eager, and bench.py's N = 2 path rehearsed (gloo, two ranks on one GPU).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
run() {  # run <name> <cmd...>: stop the whole script on a crash / timeout, continue on exit 1
  local name=$1; shift
  timeout -k 10 120 "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc: $(tail -2 gpurun_out/$name.log | tr '\n' ' ' | cut -c1-300)"
  if [ $rc -ge 124 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
run g_lg_detach env DIAG_KEEP=1 DIAG_DETACH=1 DIAG_PRE=1 python -u tools/graph_diag.py lg step
run g_simple_detach env DIAG_KEEP=1 DIAG_DETACH=1 DIAG_PRE=1 python -u tools/graph_diag.py simple step
run bench_graph python -u bench.py --graph 1 --steps 20 --warmup 3 --cpu-baseline 0 --roofline 0 --fwd-line 0
run bench_eager python -u bench.py --steps 20 --warmup 3 --cpu-baseline 0 --roofline 0 --fwd-line 0
bash tools/dp_rehearsal.sh
