#!/bin/bash
# Round 6 pre-registered from-scratch accuracy run: one batch of paired seeds from the frozen
# round-5 build in acc_frozen/ (reference side: ATen on the MI355X; ours: the HIP path).  usage:
#   bash scripts/gpu_r6_acc.sh <seeds a-b> <tag>
set -e
mkdir -p gpurun_out
cd acc_frozen
[ -e gpurun_out ] || ln -s ../gpurun_out gpurun_out
[ -e data_pack ] || ln -s ../data_pack data_pack
REFJ=12 OURJ=3 bash scripts/gpu_r5_acc.sh "$1" "$1" - - "$2" 1000
