#!/bin/bash
# Round 5: the cross-stream image Adam schedule (TSPM_ADAM_CROSS) and the audio LDS floor: bitwise tests, then A/B.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=$1
P=$PWD/task-specific-pretraining-multimodal_amd/libtspm.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py -k "schedules_equal or adam_split" -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
timeout -k 10 500 python -u scripts/ab_lib.py --rounds 3 --b $P --env-b TSPM_ADAM_CROSS=1 -- --steps 200 > gpurun_out/${T}_cross.json 2> gpurun_out/${T}_cross.err
TSPM_SLACK_LDS_FLOOR=82000 timeout -k 10 500 python -u scripts/ab_lib.py --rounds 3 --b $P --env-b TSPM_ADAM_CROSS=1 -- --steps 200 > gpurun_out/${T}_cross_floor.json 2> gpurun_out/${T}_cross_floor.err
