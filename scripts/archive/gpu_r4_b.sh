#!/bin/bash
# Round-4: fused head (tspm_head_train_step) parity + the step tests + a bench line.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r4b}
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_head.py tests/test_gpu_model.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err
timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/${T}_bench2.json 2> gpurun_out/${T}_bench2.err
