# Phase stamps of single conv launches, loader-wave build vs single-role build.
set -e
mkdir -p gpurun_out
ONLY="fwd:8,24,64,64,3,1;fwd:2,2,256,256,3,1;fwd:7,7,64,64,3,1;dgrad:8,24,64,64,3,1;wgrad:8,24,64,64,3,1;dgrad:2,2,256,256,3,1"
timeout -k 10 200 python -u scripts/stamp_conv.py --only "$ONLY" > gpurun_out/r3_stamps_loader.txt 2>&1
TSPM_LIB=$PWD/task-specific-pretraining-multimodal_amd/libtspm_stamps_noload.so timeout -k 10 200 python -u scripts/stamp_conv.py --only "$ONLY" > gpurun_out/r3_stamps_noload.txt 2>&1
