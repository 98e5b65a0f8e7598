"""Per-kernel MFMA utilisation from a tools/pmc_mfma.sh pass.

mfma_frac = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x the dispatch's cycles), the cycles taken two ways:
GRBM_GUI_ACTIVE / 8 (GPU-active cycles of one XCD; reads high on dispatches under ~0.3 ms,
MI355X_MICROARCH.md DVFS item) and the kernel-trace duration x 2.4 GHz (the nominal clock; the in-kernel
clock of these GEMMs measured 2.30-2.35 GHz in round 3, profiles/r03_gemm_clock.json).  SQ_VALU_MFMA_BUSY_CYCLES
counts 64 cycles per v_mfma_f32_32x32x2_f32, 32 per v_mfma_f32_16x16x4_f32 / v_mfma_f32_32x32x16_bf16.
"""
import csv
import glob
import os
import sys
from collections import defaultdict

d = sys.argv[1]
cnt = defaultdict(dict)
names = {}
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        did = r.get("Dispatch_Id") or r.get("Correlation_Id")
        names[did] = r["Kernel_Name"]
        cnt[did][r["Counter_Name"]] = cnt[did].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
dur = {}
for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        did = r.get("Dispatch_Id") or r.get("Correlation_Id")
        dur[did] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
agg = defaultdict(lambda: defaultdict(float))
for did, c in cnt.items():
    k = names[did]
    a = agg[k]
    a["n"] += 1
    for n, v in c.items():
        a[n] += v
    if did in dur:
        a["dur"] += dur[did]
        a["ndur"] += 1
rows = sorted(agg.items(), key=lambda kv: -kv[1].get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0))
print(f"{'kernel':58s} {'launches':>8s} {'avg_us':>8s} {'mfma_Mcyc':>10s} {'frac_grbm':>9s} {'frac_2.4GHz':>11s}")
for k, a in rows:
    mf = a.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
    if mf <= 0:
        continue
    n = a["n"]
    grbm = a.get("GRBM_GUI_ACTIVE", 0.0) / 8.0
    fg = mf / (1024.0 * grbm) if grbm else float("nan")
    avg = a["dur"] / a["ndur"] if a.get("ndur") else float("nan")
    ft = mf / (1024.0 * a["dur"] * 2.4e9) if a.get("dur") else float("nan")
    short = k.replace("(anonymous namespace)::", "").replace("void ", "").replace("hgnn::", "").split("(")[0]
    print(f"{short[:58]:58s} {n:8.0f} {avg * 1e6:8.1f} {mf / n / 1e6:10.2f} {fg:9.3f} {ft:11.3f}")
