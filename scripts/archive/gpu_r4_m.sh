#!/bin/bash
# Round-4 A/B: the head's weight-gradient launch on the image stream vs on the audio stream (same process), and
# the BN backward partial batching threshold (two libraries, alternating).
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=$1
timeout -k 10 300 python3 -u scripts/ab_step.py --variants 'side:{}' 'main:{"head_on_side":false}' --rounds 8 --k 50 > gpurun_out/${T}_ab_head.json 2> gpurun_out/${T}_ab_head.err
for i in 1 2; do
  timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/${T}_puA$i.json 2> gpurun_out/${T}_puA$i.err
  TSPM_LIB=$GRAFT_REPO_ROOT/task-specific-pretraining-multimodal_amd/libtspm_pu64.so timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/${T}_puB$i.json 2> gpurun_out/${T}_puB$i.err
done
