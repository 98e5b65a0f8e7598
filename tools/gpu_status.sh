#!/bin/bash
# Status call: GPU tests + two short benches (gpu_quick.sh), then kernel traces of the bench step
# with the side stream (gpurun_out/kt_step.txt) and with everything on the main stream
# (HGNN_SERIAL_BWD=1: standalone kernel durations, gpurun_out/kt_serial_step.txt).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_quick.sh || exit $?
SKIP_PMC=1 bash tools/prof_fused.sh > /dev/null || exit $?
head -3 gpurun_out/kt_step.txt
HGNN_SERIAL_BWD=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_serial -o run \
    -- python3 bench.py --steps 5 --warmup 2 --cpu-baseline 0 --roofline 0 --fwd-line 0 > gpurun_out/kt_serial.log 2>&1 || exit $?
f=$(find gpurun_out/kt_serial -name "*kernel_trace.csv" | head -1)
python3 tools/trace_step.py "$f" 7 > gpurun_out/kt_serial_step.txt 2>&1 || exit $?
head -3 gpurun_out/kt_serial_step.txt
