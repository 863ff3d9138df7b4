#!/bin/bash
# Alternating-process A/B of libtspm.so (A) against libtspm_alt.so (B, a build switch), batch 128 then 1024.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r6rs}
P=task-specific-pretraining-multimodal_amd
timeout -k 10 600 python -u scripts/ab_lib.py --rounds 4 --a $P/libtspm.so --b $P/libtspm_alt.so -- --steps 200 --no-cpu-baseline --pcie-steps 0 --profile-steps 0 > gpurun_out/${T}_ab_b128.json 2> gpurun_out/${T}_ab_b128.err
timeout -k 10 600 python -u scripts/ab_lib.py --rounds 3 --a $P/libtspm.so --b $P/libtspm_alt.so -- --batch-per-rank 1024 --steps 40 --no-cpu-baseline --pcie-steps 0 --profile-steps 0 > gpurun_out/${T}_ab_b1024.json 2> gpurun_out/${T}_ab_b1024.err
