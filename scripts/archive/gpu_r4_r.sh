#!/bin/bash
# per-step BN batch-statistics check of the captured step: two-level in-conv merge vs tspm_bn_finalize
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/bn_stats_check.py --steps 300 > gpurun_out/r4r_bn_stats_two_level.json 2>&1
timeout -k 10 300 python -u scripts/bn_stats_check.py --steps 300 --finalize > gpurun_out/r4r_bn_stats_finalize.json 2>&1
