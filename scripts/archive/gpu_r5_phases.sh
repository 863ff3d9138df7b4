#!/bin/bash
# Round 5: the four-phase DP exchange — its GPU tests, then the --phased line A/B against three phases.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=$1
P=$PWD/task-specific-pretraining-multimodal_amd/libtspm.so
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_model.py tests/test_gpu_ddp.py tests/test_gpu_capture.py tests/test_gpu_phased.py > gpurun_out/${T}_tests.log 2>&1
tail -3 gpurun_out/${T}_tests.log
timeout -k 10 700 python -u scripts/ab_lib.py --rounds 3 --b $P --env-b TSPM_DP_PHASES=3 -- --phased --no-cpu-baseline --pcie-steps 0 --profile-steps 0 --steps 100 > gpurun_out/${T}_ab.json 2> gpurun_out/${T}_ab.err
