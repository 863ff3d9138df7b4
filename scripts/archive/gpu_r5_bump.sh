#!/bin/bash
# Round 5: the step count / num_batches_tracked advanced at the audio chain's head and the head's weight-gradient
# launch moved behind the fork (TSPM_STEP_START_BUMP): model / head / DP tests, then A/B.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=$1
P=$PWD/task-specific-pretraining-multimodal_amd/libtspm.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_head.py tests/test_gpu_ddp.py tests/test_gpu_phased.py tests/test_gpu_harness.py tests/test_gpu_capture.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
timeout -k 10 500 python -u scripts/ab_lib.py --rounds 3 --b $P --env-b TSPM_STEP_START_BUMP=0 -- --steps 200 > gpurun_out/${T}_ab.json 2> gpurun_out/${T}_ab.err
