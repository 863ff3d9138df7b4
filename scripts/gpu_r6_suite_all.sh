#!/bin/bash
# The whole GPU suite without stopping at the first failure, then the default and batch-32 bench lines.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r6_v9}
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail 20 --timeout 300 --timeout-method thread > gpurun_out/${T}_gpu_suite.log 2>&1 || true
timeout -k 10 400 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err
timeout -k 10 200 python -u bench.py --no-cpu-baseline --pcie-steps 0 --batch-per-rank 32 --steps 50 > gpurun_out/${T}_b32.json 2> gpurun_out/${T}_b32.err
