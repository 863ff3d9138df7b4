#!/bin/bash
# Whole-step A/B of the variant-4 twins at batch 128 and 1024; each step under its own limit.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r6s3}
TUNE_BATCH=128 timeout -k 10 400 python -u scripts/split_step_ab.py profiles/r6/r6s1_split_ab_b128.json --out gpurun_out/${T}_step_ab_b128.json > gpurun_out/${T}_step_ab_b128.log 2>&1
TUNE_BATCH=1024 timeout -k 10 500 python -u scripts/split_step_ab.py profiles/r6/r6s2_split_ab_b1024.json --pairs 2 --rounds 6 --steps 10 --out gpurun_out/${T}_step_ab_b1024.json > gpurun_out/${T}_step_ab_b1024.log 2>&1
