#!/bin/bash
# Round 5: conv loader ablations (diagnostic builds, never the product): the product library, the loaders with no
# operand loads (TSPM_EXP_NOLOAD) and the loaders re-reading one stage (TSPM_EXP_SAMEADDR), graph-timed per conv.
#   bash scripts/gpu_r5_ablate.sh TAG
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=$1
P=task-specific-pretraining-multimodal_amd
ONLY="fwd:8,24,64,64,3,1;dgrad:8,24,64,64,3,1;wgrad:8,24,64,64,3,1;fwd:4,12,128,128,3,1;dgrad:4,12,128,128,3,1;wgrad:4,12,128,128,3,1;fwd:2,6,256,256,3,1;fwd:7,7,64,64,3,1;fwd:4,4,128,128,3,1;fwd:2,2,256,256,3,1"
for v in main noload sameaddr; do
  lib=$P/libtspm.so
  [ $v != main ] && lib=$P/libtspm_$v.so
  TSPM_LIB=$PWD/$lib timeout -k 10 240 python -u scripts/conv_bench.py --only "$ONLY" --json gpurun_out/${T}_$v.json > gpurun_out/${T}_$v.txt 2>&1
done
