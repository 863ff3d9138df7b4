#!/bin/bash
# batch 32: current tables (A) vs + the in-step pass (B, TSPM_TUNED_FILE), bench.py in alternating processes.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r6ab32}
P=task-specific-pretraining-multimodal_amd
timeout -k 10 600 python -u scripts/ab_lib.py --rounds 3 --a $P/libtspm.so --b $P/libtspm.so --env-b TSPM_TUNED_FILE=$GRAFT_REPO_ROOT/ab_old/tuned_b1024_pass2.json -- --batch-per-rank 1024 --steps 40 --no-cpu-baseline --pcie-steps 0 --profile-steps 0 > gpurun_out/${T}_b1024.json 2> gpurun_out/${T}_b1024.err
