"""Print one training step's kernel timeline from a rocprofv3 kernel trace CSV."""
import csv
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof/run_kernel_trace.csv"
which = int(sys.argv[2]) if len(sys.argv) > 2 else -2
rows = list(csv.DictReader(open(path)))
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Grid_Size_X"]) for r in rows)
idx = [i for i, k in enumerate(ks) if "k_plan" in k[2]]
s, e = idx[which], idx[which + 1]
t0 = ks[s][0]
tot = 0.0
for st, en, n, g in ks[s:e]:
    tot += (en - st) / 1000
    print(f"{(st - t0) / 1000:8.1f} {(en - st) / 1000:7.1f}  {n[:80]:80s} {g}")
print(f"kernel sum {tot:.1f} us, span {(ks[e][0] - t0) / 1000:.1f} us")
