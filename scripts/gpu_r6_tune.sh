#!/bin/bash
# Round 6: isolated tuning with the variant-4 kernels among the candidates, then a whole-step A/B of the tuned
# table against the current one.  usage: gpu_r6_tune.sh TAG BATCH VARIANTS
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=$1; B=$2; V=$3
timeout -k 10 600 python -u scripts/tune_convs.py --batch $B --variants $V --out gpurun_out/${T}_tuned_b$B.json > gpurun_out/${T}_tune_b$B.log 2>&1
TUNE_BATCH=$B timeout -k 10 400 python -u scripts/split_step_ab.py --table gpurun_out/${T}_tuned_b$B.json --pairs 2 --rounds 6 --steps ${STEPS:-30} --out gpurun_out/${T}_table_ab_b$B.json > gpurun_out/${T}_table_ab_b$B.log 2>&1
