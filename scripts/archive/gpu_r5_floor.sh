#!/bin/bash
# Round 5: A/B of the audio encoder's LDS floor (TSPM_SLACK_LDS_FLOOR) in the benched two-stream step.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=$1; shift
P=$PWD/task-specific-pretraining-multimodal_amd/libtspm.so
for f in "$@"; do
  timeout -k 10 500 python -u scripts/ab_lib.py --rounds 3 --b $P --env-b TSPM_SLACK_LDS_FLOOR=$f -- --steps 200 > gpurun_out/${T}_floor$f.json 2> gpurun_out/${T}_floor$f.err
done
