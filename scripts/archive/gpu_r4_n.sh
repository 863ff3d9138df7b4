#!/bin/bash
# A/B: BN statistics of the many-tile layers merged in two levels inside the conv forward (no tspm_bn_finalize
# launch) for the audio encoder only / both encoders, against the finalize launches (scripts/ab_step.py).
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u scripts/ab_step.py --rounds 8 --variants 'plain:{}' 'bn2a:{"_bn2":"a"}' \
  'bn2ai:{"_bn2":"ai"}' > gpurun_out/r4n_ab_bn2.json 2> gpurun_out/r4n_ab_bn2.err
