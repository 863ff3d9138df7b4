#!/bin/bash
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r6b2}
timeout -k 10 200 python -u scripts/split_bias.py > gpurun_out/${T}_bias.log 2>&1
timeout -k 10 300 python -u -m pytest tests/test_gpu_split.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_split_tests.log 2>&1
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py -x -q --timeout 300 --timeout-method thread -k "oracle" > gpurun_out/${T}_model.log 2>&1
