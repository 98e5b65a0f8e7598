"""Summary of a rocprofv3 --stats kernel_stats.csv under a directory: total time, calls, average per kernel.
usage: python tools/kstats.py gpurun_out/kt_dir [top]"""
import csv
import glob
import sys

f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
rows = list(csv.DictReader(open(f)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"{f}: total kernel time {tot / 1e6:.3f} ms")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
    print(f"{float(r['TotalDurationNs']) / 1e3:12.1f} us {int(r['Calls']):7d} calls {float(r['AverageNs']) / 1e3:9.2f} us avg  "
          f"{r['Name'][:110]}")
