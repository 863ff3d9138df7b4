#!/bin/bash
# Same library, current tuned tables (A) vs the tables at the start of the session (B, TSPM_TUNED_FILE), bench.py in
# alternating processes, batch 128 and 1024.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r6tab}
P=task-specific-pretraining-multimodal_amd
timeout -k 10 600 python -u scripts/ab_lib.py --rounds 4 --a $P/libtspm.so --b $P/libtspm.so --env-b TSPM_TUNED_FILE=$GRAFT_REPO_ROOT/ab_old/tuned_r6start.json -- --steps 200 --no-cpu-baseline --pcie-steps 0 --profile-steps 0 > gpurun_out/${T}_ab_b128.json 2> gpurun_out/${T}_ab_b128.err
timeout -k 10 600 python -u scripts/ab_lib.py --rounds 3 --a $P/libtspm.so --b $P/libtspm.so --env-b TSPM_TUNED_FILE=$GRAFT_REPO_ROOT/ab_old/tuned_r6start.json -- --batch-per-rank 1024 --steps 40 --no-cpu-baseline --pcie-steps 0 --profile-steps 0 > gpurun_out/${T}_ab_b1024.json 2> gpurun_out/${T}_ab_b1024.err
