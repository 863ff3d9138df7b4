#!/bin/bash
# two-level in-conv BN merge A/B at batch 1024 (scripts/ab_step.py), then one accuracy batch (gpu_r4_acc.sh)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/ab_step.py --batch 1024 --rounds 6 --k 10 --variants 'plain:{}' \
  'bn2ai:{"_bn2":"ai"}' > gpurun_out/r4o_ab_bn2_b1024.json 2> gpurun_out/r4o_ab_bn2_b1024.err
env REFJ=9 OURJ=2 PTRJ=3 PTOJ=1 bash scripts/gpu_r4_acc.sh 33-41 33-41 18-20 18-20 acc5 1000
