#!/bin/bash
# Round-4 first GPU call: baseline line on this tree, the counter list, and the MFMA-busy / LDS PMC passes
# over the batch-128 and batch-1024 benches (scripts/pmc_mfma.sh).  Each step under its own limit.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=r4a
timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err
(cd /tmp && timeout -s KILL 60 rocprofv3 -L > $GRAFT_REPO_ROOT/gpurun_out/${T}_counters.txt 2>&1) || true
bash scripts/pmc_mfma.sh ${T}_b128
bash scripts/pmc_mfma.sh ${T}_b1024 --batch-per-rank 1024
