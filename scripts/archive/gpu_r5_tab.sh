#!/bin/bash
# Round 5: the in-step retuned batch-128 table vs the table before it; the audio LDS floor and the carried Adam
# at batch 1024 (each an alternating-process A/B).
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=$1
P=$PWD/task-specific-pretraining-multimodal_amd/libtspm.so
timeout -k 10 500 python -u scripts/ab_lib.py --rounds 3 --b $P --env-b TSPM_TUNED_FILE=$PWD/scripts/tables/r5_before_instep.json -- --steps 200 > gpurun_out/${T}_table.json 2> gpurun_out/${T}_table.err
timeout -k 10 600 python -u scripts/ab_lib.py --rounds 2 --b $P --env-b TSPM_SLACK_LDS_FLOOR=0 -- --batch-per-rank 1024 --steps 30 > gpurun_out/${T}_floor_b1024.json 2> gpurun_out/${T}_floor_b1024.err
timeout -k 10 600 python -u scripts/ab_lib.py --rounds 2 --b $P --env-b TSPM_ADAM_CARRY=none -- --batch-per-rank 1024 --steps 30 > gpurun_out/${T}_carry_b1024.json 2> gpurun_out/${T}_carry_b1024.err
