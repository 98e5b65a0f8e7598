#!/bin/bash
# rocprofv3 kernel trace of one bench_configs configuration ($1, or CFG=...), per-kernel totals per step.
set -u
set -- "${1:-${CFG:-cfg1g}}"
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_$1 -o run \
    -- python3 tools/bench_configs.py --only $1 --steps ${STEPS:-10} --warmup 3 > gpurun_out/kt_$1.log 2>&1
rc=$?; echo "kt rc=$rc"; [ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/kt_$1 -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total kernel time {tot/1e6:.2f} ms")
for r in rows[:25]:
    n = r["Name"].replace("(anonymous namespace)::", "").replace("void ", "").replace("hgnn::", "").split("(")[0]
    print(f'{float(r["TotalDurationNs"])/1e3:10.1f} us {int(r["Calls"]):6d} calls {float(r["AverageNs"])/1e3:8.2f} us avg  {n[:70]}')
PY
