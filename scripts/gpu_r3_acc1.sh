# Accuracy parity, scratch config: concurrent seeds on one GPU.
set -e
export MIOPEN_FIND_MODE=FAST
mkdir -p gpurun_out
timeout -k 10 330 python -u scripts/acc_par.py --jobs 4 --limit 300 --deadline 240 -- ours --epochs 20 --seeds 0-95 > gpurun_out/acc1_ours.log 2>&1
timeout -k 10 800 python -u scripts/acc_par.py --jobs 8 --limit 700 --deadline 420 -- reference --device cuda --epochs 20 --seeds 0-95 > gpurun_out/acc1_ref.log 2>&1
