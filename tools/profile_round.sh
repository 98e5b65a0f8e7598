#!/bin/bash
# The round's profile set, copied under profiles/ by the caller (prefix $R, e.g. r02):
#   1. kernel trace + stats of the headline bench (per-kernel time per step)
#   2. PMC HBM traffic of every bench kernel (FETCH_SIZE and WRITE_SIZE in separate passes)
#   3. SQ wave states of the bench kernels (one PMC pass)
#   4. kernel stats + PMC traffic of the CCN configurations (cfg3 CCN-1D, cfg5 CCN-2D)
#   5. every bench_configs.py configuration (JSON lines, CCN lines with their roofline object)
# Each step has its own time limit; the first failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
SKIP_PMC=1 bash tools/prof_fused.sh || exit $?
bash tools/pmc.sh > /dev/null || exit $?
echo "pmc traffic ok"
C="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS"
timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d gpurun_out/pmc_sq -o run \
    -- python3 bench.py --steps 3 --warmup 2 --settle-s 0 --attribution 0 --cpu-baseline 0 --roofline 0 --fwd-line 0 > gpurun_out/pmc_sq.log 2>&1 || exit $?
python3 tools/pmc_sq_summary.py gpurun_out/pmc_sq > gpurun_out/pmc_sq_summary.txt || exit $?
echo "pmc sq ok"
for cfg in cfg3 cfg5; do
  STEPS=6 bash tools/prof_cfg.sh $cfg > gpurun_out/kt_${cfg}_summary.txt || exit $?
  for P in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 200 rocprofv3 --pmc $P --kernel-trace --output-format csv -d gpurun_out/pmc_${cfg}_$P -o run \
        -- python3 tools/bench_configs.py --only $cfg --steps 4 --warmup 2 > gpurun_out/pmc_${cfg}_$P.log 2>&1 || exit $?
  done
  python3 tools/pmc_summary.py gpurun_out/pmc_${cfg}_FETCH_SIZE gpurun_out/pmc_${cfg}_WRITE_SIZE gpurun_out/pmc_${cfg}_traffic.json \
      > gpurun_out/pmc_${cfg}_summary.txt || exit $?
  echo "$cfg ok"
done
timeout -k 10 600 python3 tools/bench_configs.py > gpurun_out/configs.jsonl 2> gpurun_out/configs.err || exit $?
echo "configs ok"
