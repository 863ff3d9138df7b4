#!/bin/bash
# Round 5: the single-launch BN backward for the few-row layers (k_bn_bwd_small): BN / model tests, then A/B.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=$1
P=$PWD/task-specific-pretraining-multimodal_amd/libtspm.so
timeout -k 10 500 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_bn_src.py tests/test_gpu_bn_pool.py tests/test_gpu_model.py tests/test_gpu_mono.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
timeout -k 10 500 python -u scripts/ab_lib.py --rounds 3 --b $P --env-b TSPM_BN_SMALL_ROWS=0 -- --steps 200 > gpurun_out/${T}_ab.json 2> gpurun_out/${T}_ab.err
