#!/bin/bash
# Config 5 (CCN-2D, 64 SBM-200 graphs): kernel trace + two SQ counter passes (wave states / instruction mix,
# LDS), each pass its own run with its own limit.  Output under gpurun_out/cfg5_*.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=6 bash tools/prof_cfg.sh cfg5 > gpurun_out/cfg5_kt.txt || exit $?
cat gpurun_out/cfg5_kt.txt | head -14
C1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD"
timeout -s KILL 200 rocprofv3 --pmc $C1 --kernel-trace --output-format csv -d gpurun_out/cfg5_sq1 -o run \
    -- python3 tools/bench_configs.py --only cfg5 --steps 3 --warmup 1 > gpurun_out/cfg5_sq1.log 2>&1 || exit $?
python3 tools/pmc_sq_summary.py gpurun_out/cfg5_sq1 | head -12
C2="SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
timeout -s KILL 200 rocprofv3 --pmc $C2 --kernel-trace --output-format csv -d gpurun_out/cfg5_sq2 -o run \
    -- python3 tools/bench_configs.py --only cfg5 --steps 3 --warmup 1 > gpurun_out/cfg5_sq2.log 2>&1 || exit $?
python3 - <<'PY'
import csv, glob, os
from collections import defaultdict
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob("gpurun_out/cfg5_sq2/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, c in sorted(acc.items(), key=lambda kv: -sum(kv[1].get("SQ_WAVE_CYCLES", [0]))):
    m = {n: sum(v) / len(v) for n, v in c.items()}
    w = max(m.get("SQ_WAVES", 1), 1)
    short = k.replace("(anonymous namespace)::", "").replace("void ", "").replace("hgnn::", "").split("(")[0]
    print(f"{short[:45]:45s} lds/w {m.get('SQ_INSTS_LDS',0)/w:8.1f} smem/w {m.get('SQ_INSTS_SMEM',0)/w:7.1f} "
          f"bank_confl/idx_active {m.get('SQ_LDS_BANK_CONFLICT',0)/max(m.get('SQ_LDS_IDX_ACTIVE',1),1):.3f} "
          f"wait_lds/wave_cyc {m.get('SQ_WAIT_INST_LDS',0)/max(m.get('SQ_WAVE_CYCLES',1),1):.3f}")
    if "k_c2" not in k and "ccn2" not in k:
        break
PY
