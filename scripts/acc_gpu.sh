set -e
export MIOPEN_FIND_MODE=FAST
mkdir -p gpurun_out
timeout -k 10 450 python -u scripts/accuracy_parity.py ours --epochs 20 --seeds 0,1,2,3,4,5,6,7 > gpurun_out/acc_ours.log 2>&1
timeout -k 10 650 python -u scripts/accuracy_parity.py reference --device cuda --epochs 20 --seeds 0,1,2,3,4,5,6,7 > gpurun_out/acc_refgpu.log 2>&1
