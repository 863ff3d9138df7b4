#!/bin/bash
# A/B: the one-thread launches (step-count increment, num_batches_tracked) moved off the audio chain
# (FusedTrainStep lean_tail) against the committed schedule, batch 128 and 1024 (scripts/ab_step.py)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/ab_step.py --rounds 10 --variants 'plain:{}' 'lean:{"lean_tail":true}' \
  > gpurun_out/r4q_ab_lean.json 2> gpurun_out/r4q_ab_lean.err
timeout -k 10 300 python -u scripts/ab_step.py --batch 1024 --rounds 6 --k 10 --variants 'plain:{}' \
  'lean:{"lean_tail":true}' > gpurun_out/r4q_ab_lean_b1024.json 2> gpurun_out/r4q_ab_lean_b1024.err
[ -n "$ACC" ] && env REFJ=10 OURJ=3 PTRJ=1 PTOJ=1 bash scripts/gpu_r4_acc.sh 52-61 52-61 22 22 acc7 1000
exit 0
