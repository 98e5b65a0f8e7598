#!/bin/bash
# Round 6: switch / off-diagonal tests, then kernel + memory-copy traces of the forced RCCL world-1 bench and of the
# plain bench (CSV, for the per-stream gap analysis of tools/trace_gaps.py).
set -u
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_switches.py "tests/test_gpu_net.py::test_offdiagonal_identity_or_degree_slice_raises" -x -q --timeout 250 --timeout-method thread > gpurun_out/t1.log 2>&1
rc=$?; tail -3 gpurun_out/t1.log; [ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
cd /tmp
for mode in dp plain; do
  if [ $mode = dp ]; then X="--force-dp 1"; else X=""; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $R/gpurun_out/tr_$mode -o run -- python3 $R/bench.py --cpu-baseline 0 --roofline 0 --fwd-line 0 --attribution 0 --settle-s 0.3 --steps 20 $X > $R/gpurun_out/tr_$mode.log 2>&1
  rc=$?; echo "trace $mode rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
