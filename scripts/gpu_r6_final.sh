#!/bin/bash
# Round-6 evidence set on the committed tree, in two calls (each under gpurun's 20-minute limit):
#   bash scripts/gpu_r6_final.sh suite TAG   smoke + the whole GPU suite
#   bash scripts/gpu_r6_final.sh prof  TAG   the headline line + rocprofv3 stats / trace + PMC FETCH / WRITE passes
#                                            (scripts/prof_bench.sh), the MFMA-busy passes at batch 128 and 1024
#                                            (scripts/pmc_mfma.sh)
#   bash scripts/gpu_r6_final.sh lines TAG   the other BASELINE configs' lines, --phased
# Each step has its own time limit; the script stops at the first failure.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
MODE=$1
T=${2:-r6_v1}
if [ "$MODE" = "suite" ]; then
  timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_gpu_suite.log 2>&1
  exit 0
fi
if [ "$MODE" = "prof" ]; then
  bash scripts/prof_bench.sh $T
  bash scripts/pmc_mfma.sh ${T}_b128
  bash scripts/pmc_mfma.sh ${T}_b1024 --batch-per-rank 1024
  exit 0
fi
timeout -k 10 300 python -u bench.py --kernel-table gpurun_out/${T}_kernel_table.json > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err
timeout -k 10 200 python -u bench.py --no-cpu-baseline --pcie-steps 0 --batch-per-rank 32 --steps 50 > gpurun_out/${T}_bench_b32.json 2> gpurun_out/${T}_b32.err
timeout -k 10 300 python -u bench.py --no-cpu-baseline --pcie-steps 0 --batch-per-rank 1024 --steps 20 --kernel-table gpurun_out/${T}_kernel_table_b1024.json > gpurun_out/${T}_bench_b1024.json 2> gpurun_out/${T}_b1024.err
timeout -k 10 200 python -u bench.py --mono > gpurun_out/${T}_mono.json 2> gpurun_out/${T}_mono.err
timeout -k 10 200 python -u bench.py --mmimdb > gpurun_out/${T}_mmimdb.json 2> gpurun_out/${T}_mmimdb.err
timeout -k 10 200 python -u bench.py --mosi > gpurun_out/${T}_mosi.json 2> gpurun_out/${T}_mosi.err
timeout -k 10 200 python -u bench.py --mosi --mosei > gpurun_out/${T}_mosei.json 2> gpurun_out/${T}_mosei.err
timeout -k 10 200 python -u bench.py --phased --no-cpu-baseline --pcie-steps 0 --profile-steps 0 --steps 100 > gpurun_out/${T}_phased.json 2> gpurun_out/${T}_phased.err
