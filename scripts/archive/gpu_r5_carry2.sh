#!/bin/bash
# Round 5: carried-Adam variants, each A/B against the plain schedule (alternating processes).
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=$1; shift
P=$PWD/task-specific-pretraining-multimodal_amd/libtspm.so
for v in "$@"; do
  timeout -k 10 500 python -u scripts/ab_lib.py --rounds 3 --b $P --env-b $v -- --steps 200 > "gpurun_out/${T}_$v.json" 2> "gpurun_out/${T}_$v.err"
done
