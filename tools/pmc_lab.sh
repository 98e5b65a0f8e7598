#!/bin/bash
# One PMC pass over the GEMM lab: effective clock (GRBM_GUI_ACTIVE / 8 / wall), MFMA busy and wave states.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_BUSY_CYCLES \
    --output-format csv -d gpurun_out/pmc_lab -o run -- ./tools/${LAB:-gemm4_lab} > gpurun_out/pmc_lab.log 2>&1
rc=$?; echo "pmc rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/pmc_lab.log; exit $rc; }
python3 - <<'PY'
import csv, collections, glob
f = glob.glob('gpurun_out/pmc_lab/**/*counter_collection.csv', recursive=True)[0]
d = collections.defaultdict(dict)
for r in csv.DictReader(open(f)):
    k = r['Dispatch_Id']
    d[k][r['Counter_Name']] = float(r['Counter_Value'])
    d[k]['name'] = r['Kernel_Name'].split('(')[0].replace('void ', '')[:40]
    d[k]['dur'] = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
    d[k]['grid'] = r['Grid_Size']
agg = collections.OrderedDict()
for k in sorted(d, key=int):
    v = d[k]
    key = (v['name'], v['grid'])
    agg.setdefault(key, []).append(v)
print(f"{'kernel':40s} {'grid':>8s} {'n':>3s} {'us':>7s} {'GHz':>5s} {'mfma%':>6s} {'wait':>5s} {'stall':>5s} {'lds':>5s} {'act':>5s}")
for (n, g), vs in agg.items():
    if 'k_ref' in n:
        continue
    vs = vs[1:] if len(vs) > 1 else vs
    m = lambda c: sum(x.get(c, 0) for x in vs) / len(vs)
    dur = m('dur')
    ghz = m('GRBM_GUI_ACTIVE') / 8 / (dur * 1e3)
    mf = m('SQ_VALU_MFMA_BUSY_CYCLES') / (1024 * dur * 1e3 * ghz) if ghz > 0 else 0
    wc = m('SQ_WAVE_CYCLES') or 1
    print(f"{n:40s} {g:>8s} {len(vs):3d} {dur:7.1f} {ghz:5.2f} {100*mf:6.1f} {m('SQ_WAIT_ANY')/wc:5.2f} {m('SQ_WAIT_INST_ANY')/wc:5.2f} {m('SQ_WAIT_INST_LDS')/wc:5.2f} {m('SQ_ACTIVE_INST_ANY')/wc:5.2f}")
PY
