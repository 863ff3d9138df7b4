#!/bin/bash
# Round 5: the five-phase DP exchange (TSPM_DP_PHASES=5): DP / capture tests, then an A/B of the --phased line.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=$1
P=$PWD/task-specific-pretraining-multimodal_amd/libtspm.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_capture.py tests/test_gpu_phased.py tests/test_gpu_ddp.py "tests/test_gpu_model.py::test_phased_allreduce_step_equals_plain_step" -x -q -s --timeout 300 --timeout-method thread > gpurun_out/${T}_dp_tests.log 2>&1
timeout -k 10 600 python -u scripts/ab_lib.py --rounds 3 --b $P --env-b TSPM_DP_PHASES=5 -- --phased --steps 100 --profile-steps 0 > gpurun_out/${T}_phases.json 2> gpurun_out/${T}_phases.err
