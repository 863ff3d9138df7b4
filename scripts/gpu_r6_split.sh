#!/bin/bash
# Round-6 variant-4 (bf16-piece products) validation and per-launch A/B; each step under its own limit.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r6s1}
#timeout -k 10 300 python -u -m pytest tests/test_gpu_split.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_split_tests.log 2>&1
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -k "test_conv_fwd or test_conv_dgrad or test_conv_wgrad" > gpurun_out/${T}_ops_v4.log 2>&1
timeout -k 10 400 python -u scripts/split_ab.py --json gpurun_out/${T}_split_ab.json > gpurun_out/${T}_split_ab.log 2>&1
