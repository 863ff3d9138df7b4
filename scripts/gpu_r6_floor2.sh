#!/bin/bash
# Audio LDS floor re-measured on the final tables: default 82000 (A) vs 0 and 54000 (B runs).
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r6fl}
P=task-specific-pretraining-multimodal_amd
timeout -k 10 500 python -u scripts/ab_lib.py --rounds 4 --a $P/libtspm.so --b $P/libtspm.so --env-b TSPM_SLACK_PARTS=f -- --steps 200 --no-cpu-baseline --pcie-steps 0 --profile-steps 0 > gpurun_out/${T}_f.json 2> gpurun_out/${T}_f.err
