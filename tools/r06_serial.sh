#!/bin/bash
# stamp timeline of the step, then a kernel trace with every backward kernel on the main stream (standalone durations)
set -u
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python tools/timeline.py --steps 6 --json gpurun_out/tl.json > gpurun_out/timeline.txt 2>&1 || { tail -5 gpurun_out/timeline.txt; exit 1; }
tail -32 gpurun_out/timeline.txt
export TMPDIR=/tmp
cd /tmp
HGNN_SERIAL_BWD=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/tr_serial -o run -- python3 $R/bench.py --cpu-baseline 0 --roofline 0 --fwd-line 0 --attribution 0 --settle-s 0.3 --steps 20 > $R/gpurun_out/tr_serial.log 2>&1
rc=$?; echo "serial trace rc=$rc"; exit $rc
