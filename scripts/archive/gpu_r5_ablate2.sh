#!/bin/bash
# Round 5: where the LDS conv's time goes (diagnostic builds, never the product).  (1) graph-timed convs: product
# library vs no-MFMA compute waves; (2) phase stamps of the audio layer-1 forward (tuned and two other tilings) and
# dgrad: stamped product build vs no operand loads vs no MFMA.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=$1
P=$PWD/task-specific-pretraining-multimodal_amd
ONLY="fwd:8,24,64,64,3,1;dgrad:8,24,64,64,3,1;wgrad:8,24,64,64,3,1;fwd:4,12,128,128,3,1;fwd:7,7,64,64,3,1;fwd:2,2,256,256,3,1"
TSPM_LIB=$P/libtspm_nomfma.so timeout -k 10 240 python -u scripts/conv_bench.py --only "$ONLY" > gpurun_out/${T}_nomfma.txt 2>&1
for v in "" _noload _nomfma; do
  TSPM_LIB=$P/libtspm_stamps$v.so timeout -k 10 240 python -u scripts/stamp_conv.py --only "fwd:8,24,64,64,3,1" --algo "2,1,1,4,1,1/2,1,2,2,1,1/1,1,2,2,1,1/1,1,1,4,1,1" > gpurun_out/${T}_stamps$v.txt 2>&1
  TSPM_LIB=$P/libtspm_stamps$v.so timeout -k 10 240 python -u scripts/stamp_conv.py --only "dgrad:8,24,64,64,3,1;fwd:4,12,128,128,3,1" >> gpurun_out/${T}_stamps$v.txt 2>&1
done
