#!/bin/bash
# Round-end verification of the committed tree: GPU tests, smoke, default bench line.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
{
  echo "== pytest -m gpu"
  timeout -k 10 500 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread 2>&1 | grep -v amdgpu.ids | tail -3
  echo "== smoke"
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | grep -v amdgpu.ids | tail -2
  echo "== bench (defaults)"
  timeout -k 10 600 python bench.py 2> gpurun_out/fv_bench.err | tail -1 | tee gpurun_out/fv_bench.json | python3 -c "
import json,sys
d=json.loads(sys.stdin.read())
print('value', d['value'], d['unit'], 'ms_per_step', d['ms_per_step'], 'settle_steps', d.get('settle_steps'))
print('roofline', {k: d['roofline'][k] for k in ('kernel','bound','achieved','peak','unit','frac','traffic')})
print('parity', d['parity']['pass'], 'cpu_baseline', d['cpu_baseline']['value'], d['cpu_baseline']['unit'])
print('attribution', d.get('attribution'))"
} > gpurun_out/final_verify.log 2>&1
cat gpurun_out/final_verify.log
