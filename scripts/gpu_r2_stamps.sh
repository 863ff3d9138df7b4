# Phase stamps of the image encoder's small forward launches (R34 layer1..4 3x3, batch 128) and a layer3 dgrad.
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/stamp_conv.py --only "fwd:7,7,64,64,3,1;fwd:4,4,128,128,3,1;fwd:2,2,256,256,3,1;fwd:1,1,512,512,3,1;dgrad:2,2,256,256,3,1" > gpurun_out/stamps_r2.log 2>&1
