"""Per-kernel averages of the SQ counters of one rocprofv3 PMC pass (tools/pmc_sq.sh).

SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles (MI355X_MICROARCH.md);
WAIT_ANY (parked in s_waitcnt / barrier) + WAIT_INST_ANY (issue stall) + ACTIVE_INST_ANY
~= WAVE_CYCLES.  Printed as fractions of WAVE_CYCLES, and instructions per wave.
"""
import csv
import glob
import os
import sys
from collections import defaultdict

d = sys.argv[1]
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
rows = []
for k, c in acc.items():
    m = {n: sum(v) / len(v) for n, v in c.items()}
    rows.append((m.get("SQ_WAVE_CYCLES", 0.0), k, m))
rows.sort(reverse=True)
print(f"{'kernel':60s} {'waves':>8s} {'wait':>6s} {'stall':>6s} {'active':>6s} {'valu/w':>7s} {'salu/w':>7s} {'vmem/w':>7s}")
for wc, k, m in rows[:25]:
    w = max(m.get("SQ_WAVES", 1.0), 1.0)
    f = lambda n: m.get(n, 0.0) / wc if wc else 0.0  # noqa: E731
    short = k.replace("(anonymous namespace)::", "").replace("void ", "").replace("hgnn::", "").split("(")[0]
    print(f"{short[:60]:60s} {w:8.0f} {f('SQ_WAIT_ANY'):6.2f} {f('SQ_WAIT_INST_ANY'):6.2f} {f('SQ_ACTIVE_INST_ANY'):6.2f} "
          f"{m.get('SQ_INSTS_VALU', 0) / w:7.1f} {m.get('SQ_INSTS_SALU', 0) / w:7.1f} {m.get('SQ_INSTS_VMEM_RD', 0) / w:7.1f}")
