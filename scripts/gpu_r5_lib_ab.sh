#!/bin/bash
# Round 5: a kernel change built as libtspm_alt.so — its GPU tests (given as pytest args after the tag),
# then a step A/B against libtspm.so (alternating processes, 3 rounds).
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=$1; shift
ALT=$PWD/task-specific-pretraining-multimodal_amd/libtspm_alt.so
TSPM_LIB=$ALT timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread "$@" > gpurun_out/${T}_tests.log 2>&1
tail -3 gpurun_out/${T}_tests.log
timeout -k 10 500 python -u scripts/ab_lib.py --rounds 3 -- --steps 200 > gpurun_out/${T}_ab.json 2> gpurun_out/${T}_ab.err
cat gpurun_out/${T}_ab.json
