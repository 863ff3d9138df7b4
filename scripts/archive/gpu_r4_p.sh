#!/bin/bash
# the model-level GPU parity tests on the two-level in-conv BN merge default, then one accuracy batch
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_mono.py -x -q --timeout 200 \
  --timeout-method thread > gpurun_out/r4p_model_tests.log 2>&1
env REFJ=10 OURJ=3 PTRJ=1 PTOJ=1 bash scripts/gpu_r4_acc.sh 42-51 42-51 21 21 acc6 1000
