#!/bin/bash
# Monomodal (ResNet18 audio, batch 256): isolated tune over variants 2 and 4, then bench --mono current vs tuned.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out ab_old
T=${1:-r6mt}
P=task-specific-pretraining-multimodal_amd
timeout -k 10 600 python -u scripts/tune_convs.py --batch 256 --encoders audio --variants 2,4 --out gpurun_out/${T}_tuned_b256.json > gpurun_out/${T}_tune_b256.log 2>&1
python scripts/merge_tuned.py ab_old/tuned_mono_new.json gpurun_out/${T}_tuned_b256.json > gpurun_out/${T}_merge.log
timeout -k 10 600 python -u scripts/ab_lib.py --rounds 4 --a $P/libtspm.so --b $P/libtspm.so --env-b TSPM_TUNED_FILE=$GRAFT_REPO_ROOT/ab_old/tuned_mono_new.json -- --mono --steps 100 > gpurun_out/${T}_ab_mono.json 2> gpurun_out/${T}_ab_mono.err
