#!/bin/bash
# Variant-4 twins for the monomodal (batch 256) table: per-launch A/B, then bench --mono current vs twins.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out ab_old
T=${1:-r6m}
P=task-specific-pretraining-multimodal_amd
timeout -k 10 500 python -u scripts/split_ab.py --batch 256 --json gpurun_out/${T}_split_ab_b256.json > gpurun_out/${T}_split_ab_b256.log 2>&1
python scripts/twin_table.py gpurun_out/${T}_split_ab_b256.json ab_old/tuned_mono_twins.json > gpurun_out/${T}_twins.log
timeout -k 10 600 python -u scripts/ab_lib.py --rounds 4 --a $P/libtspm.so --b $P/libtspm.so --env-b TSPM_TUNED_FILE=$GRAFT_REPO_ROOT/ab_old/tuned_mono_twins.json -- --mono --steps 100 > gpurun_out/${T}_ab_mono.json 2> gpurun_out/${T}_ab_mono.err
