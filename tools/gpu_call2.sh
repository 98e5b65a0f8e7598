set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 600 python tools/bench_configs.py > gpurun_out/configs.jsonl 2> gpurun_out/configs.err
rc=$?; echo "configs rc=$rc"; cat gpurun_out/configs.jsonl; tail -3 gpurun_out/configs.err
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/pmc.sh
