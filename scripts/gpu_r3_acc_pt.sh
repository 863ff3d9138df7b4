# Accuracy parity, pretrained-encoder config with the reference's ONE-group optimizer:
# reference side (ATen oracle) and ours concurrently on one GPU, 16 seeds.
set -e
export MIOPEN_FIND_MODE=FAST
mkdir -p gpurun_out
timeout -k 10 1100 python -u scripts/acc_par.py --jobs 6 --limit 1050 --deadline 560 -- pt_reference --device cuda --mono-epochs 10 --epochs 20 --seeds 0-15 > gpurun_out/accpt_ref.log 2>&1 &
P1=$!
timeout -k 10 700 python -u scripts/acc_par.py --jobs 2 --limit 650 --deadline 450 -- pt_ours --mono-epochs 10 --epochs 20 --seeds 0-15 > gpurun_out/accpt_ours.log 2>&1 &
P2=$!
wait $P1
wait $P2
