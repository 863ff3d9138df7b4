#!/bin/bash
# Stage-pair build (libtspm_alt.so, -DTSPM_SPLIT_PAIR=1): variant-4 kernel tests on it, then the step A/B.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r6p}
P=task-specific-pretraining-multimodal_amd
TSPM_LIB=$GRAFT_REPO_ROOT/$P/libtspm_alt.so timeout -k 10 300 python -u -m pytest tests/test_gpu_split.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_split_tests.log 2>&1
TSPM_LIB=$GRAFT_REPO_ROOT/$P/libtspm_alt.so timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -k "test_conv_fwd or test_conv_dgrad or test_conv_wgrad" > gpurun_out/${T}_ops.log 2>&1
bash scripts/gpu_r6_rs.sh ${T}
