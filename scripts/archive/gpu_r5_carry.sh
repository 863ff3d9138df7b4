#!/bin/bash
# Round 5: Adam updates carried by later backward launches (TSPM_ADAM_CARRY): bitwise schedule tests, then A/B.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=$1; shift
P=$PWD/task-specific-pretraining-multimodal_amd/libtspm.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py -k "schedules" -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
for v in "$@"; do
  timeout -k 10 500 python -u scripts/ab_lib.py --rounds 3 --b $P --env-b TSPM_ADAM_CARRY=$v -- --steps 200 > gpurun_out/${T}_carry_$v.json 2> gpurun_out/${T}_carry_$v.err
done
