cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ccn.py -v --timeout 200 --timeout-method thread -k "wide or degree_above or sbm200 or batched" > gpurun_out/t_wide.log 2>&1; grep -E "PASS|FAIL|Error" gpurun_out/t_wide.log | cut -c1-150
