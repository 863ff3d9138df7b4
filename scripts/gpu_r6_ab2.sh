#!/bin/bash
# (1) current tables (A) vs + in-step pass 2 (B, TSPM_TUNED_FILE) at batch 128; (2) libtspm.so vs libtspm_alt.so.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r6ab2}
P=task-specific-pretraining-multimodal_amd
timeout -k 10 600 python -u scripts/ab_lib.py --rounds 4 --a $P/libtspm.so --b $P/libtspm.so --env-b TSPM_TUNED_FILE=$GRAFT_REPO_ROOT/ab_old/tuned_pass4.json -- --steps 200 --no-cpu-baseline --pcie-steps 0 --profile-steps 0 > gpurun_out/${T}_pass4_b128.json 2> gpurun_out/${T}_pass4_b128.err

